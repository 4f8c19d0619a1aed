// Latency of one wave's accesses to fine-grained (coherent, mapped) host
// memory on MI355X, timed inside the wave with s_memrealtime (100 MHz):
// what the resident zp_parse_one server pays per dependent step.
//   hostmem_probe            (prints one line per pattern: median / p90 in us)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define G __attribute__((address_space(1)))
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

enum { P_SYS8_ONE = 0, P_NT16_WAVE, P_PLAIN16_WAVE, P_SYS8x2_WAVE, P_SYS16_WAVE_ASM,
       P_STORE8_SYS_WAIT, P_STORE8_NT_WAIT, P_DEV16_WAVE, P_STORE8_DEV_WAIT, P_NT16_WAVE_X2,
       P_COUNT };
static const char* names[P_COUNT] = {
    "1 lane, 8-B system-scope load (host)",
    "64 lanes, 16-B nt load = 1 KiB (host)",
    "64 lanes, 16-B plain load = 1 KiB (host)",
    "64 lanes, 2 x 8-B system-scope loads = 1 KiB (host)",
    "64 lanes, 16-B sc0 sc1 load (asm) = 1 KiB (host)",
    "1 lane, 8-B system-scope store + vmcnt(0) (host)",
    "64 lanes, 8-B nt store + vmcnt(0) (host)",
    "64 lanes, 16-B nt load = 1 KiB (device HBM)",
    "64 lanes, 8-B nt store + vmcnt(0) (device HBM)",
    "64 lanes, 2 x 16-B nt loads = 2 KiB (host)",
};

__global__ void __launch_bounds__(64) probe(uint8_t* h, uint8_t* d, int pat, int reps,
                                            uint64_t* out) {
    const int lane = threadIdx.x;
    uint32_t sink = 0;
    for (int r = 0; r < reps; ++r) {
        const uint32_t off = (uint32_t)(r & 7) * 4096u;   // rotate over 8 pages
        __builtin_amdgcn_s_waitcnt(0);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        switch (pat) {
        case P_SYS8_ONE:
            if (lane == 0) sink += (uint32_t)__hip_atomic_load((const G uint64_t*)(h + off),
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        case P_NT16_WAVE: {
            u32x4 v = __builtin_nontemporal_load((const G u32x4*)(h + off) + lane);
            sink += v.x ^ v.w;
        } break;
        case P_PLAIN16_WAVE: {
            u32x4 v = *((const G u32x4*)(h + off) + lane);
            sink += v.x ^ v.w;
        } break;
        case P_SYS8x2_WAVE: {
            const G uint64_t* p = (const G uint64_t*)(h + off) + 2 * lane;
            uint64_t a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            uint64_t b = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            sink += (uint32_t)(a ^ b);
        } break;
        case P_SYS16_WAVE_ASM: {
            u32x4 v;
            const G u32x4* p = (const G u32x4*)(h + off) + lane;
            asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(p) : "memory");
            sink += v.x ^ v.w;
        } break;
        case P_STORE8_SYS_WAIT:
            if (lane == 0)
                __hip_atomic_store((G uint64_t*)(h + 65536 + off), (uint64_t)r, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            break;
        case P_STORE8_NT_WAIT:
            __builtin_nontemporal_store((uint64_t)r, (G uint64_t*)(h + 65536 + off) + lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            break;
        case P_DEV16_WAVE: {
            u32x4 v = __builtin_nontemporal_load((const G u32x4*)(d + (uint64_t)r * 65536u) + lane);
            sink += v.x ^ v.w;
        } break;
        case P_STORE8_DEV_WAIT:
            __builtin_nontemporal_store((uint64_t)r, (G uint64_t*)(d + (uint64_t)r * 65536u) + lane);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            break;
        case P_NT16_WAVE_X2: {
            u32x4 v = __builtin_nontemporal_load((const G u32x4*)(h + off) + lane);
            u32x4 w = __builtin_nontemporal_load((const G u32x4*)(h + off + 1024) + lane);
            sink += v.x ^ w.w;
        } break;
        }
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(sink) :: "memory");
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) out[r] = t1 - t0;
    }
    if (sink == 0x12345678u) out[reps] = sink;
}

int main() {
    uint8_t *h = nullptr, *hd = nullptr, *d = nullptr;
    uint64_t* out = nullptr;
    const int reps = 400;
    if (hipHostMalloc((void**)&h, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostGetDevicePointer((void**)&hd, h, 0) || hipMalloc(&d, (size_t)reps * 65536 + 4096) ||
        hipMalloc(&out, (reps + 1) * 8)) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    int khz = 0;
    (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
    for (int pat = 0; pat < P_COUNT; ++pat) {
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, hd, d, pat, reps, out);
        if (hipDeviceSynchronize()) { fprintf(stderr, "kernel failed\n"); return 1; }
        std::vector<uint64_t> t(reps);
        (void)hipMemcpy(t.data(), out, reps * 8, hipMemcpyDeviceToHost);
        std::vector<double> us;
        for (int r = 20; r < reps; ++r) us.push_back(t[r] * 1000.0 / khz);
        std::sort(us.begin(), us.end());
        printf("%-55s median %6.2f us  p10 %6.2f  p90 %6.2f\n", names[pat], us[us.size() / 2],
               us[us.size() / 10], us[us.size() * 9 / 10]);
    }
    return 0;
}
