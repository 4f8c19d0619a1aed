// Doorbell round trip of a resident server wave, by where the request lives
// (lab probe for zp_parse_one's transport, not product code):
//   host:   doorbell + frame in mapped, coherent pinned host memory (the
//           product's block; the wave reads them over the host link)
//   device: doorbell + frame in fine-grained device memory the host writes
//           through its mapping (posted writes); the wave reads local HBM
// The answer always goes to host memory. Host side: write the frame, ring,
// spin on the acknowledgement; median / p90 / p99 of 4000 round trips.
//   devmem_doorbell [frame_bytes]
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <algorithm>
#include <vector>

#define G __attribute__((address_space(1)))
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(64) server(uint8_t* req, uint8_t* ack, uint32_t len) {
    const int lane = threadIdx.x;
    uint32_t seq = 0;
    for (;;) {
        uint64_t b = 0;
        if (lane == 0)
            b = __hip_atomic_load((const uint64_t*)req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t bs = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(b >> 32), 0);
        if (bs == 0xFFFFFFFFu) break;
        if (bs == seq) { __builtin_amdgcn_s_sleep(1); continue; }
        seq = bs;
        uint32_t acc = 0;
        for (uint32_t o = 16u * lane; o < len; o += 1024u) {
            u32x4 v;
            const G u32x4* p = (const G u32x4*)(req + 64 + o);
            asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n s_waitcnt vmcnt(0)"
                         : "=v"(v) : "v"(p) : "memory");
            acc += v.x ^ v.w;
        }
        for (int s = 32; s; s >>= 1) acc += __shfl_xor(acc, s);
        if (lane == 0)
            __hip_atomic_store((uint64_t*)ack, ((uint64_t)seq << 32) | acc, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static sigjmp_buf jb;
static void on_segv(int) { siglongjmp(jb, 1); }

static int64_t now_ns() {
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (int64_t)t.tv_sec * 1000000000 + t.tv_nsec;
}

static void run(const char* name, uint8_t* req_h, uint8_t* req_d, uint8_t* ack_h, uint8_t* ack_d,
                uint32_t len) {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    memset(ack_h, 0, 8);
    __atomic_store_n((uint64_t*)req_h, (uint64_t)0, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(server, dim3(1), dim3(64), 0, s, req_d, ack_d, len);
    std::vector<uint8_t> frame(len);
    for (uint32_t i = 0; i < len; ++i) frame[i] = (uint8_t)(i * 7 + 1);
    std::vector<double> us;
    for (uint32_t k = 1; k <= 4200; ++k) {
        frame[0] = (uint8_t)k;
        const int64_t t0 = now_ns();
        memcpy(req_h + 64, frame.data(), len);
        _mm_sfence();                        // device memory is write-combined on the host
        __atomic_store_n((uint64_t*)req_h, (uint64_t)k << 32, __ATOMIC_RELEASE);
        _mm_sfence();
        while ((uint32_t)(__atomic_load_n((volatile uint64_t*)ack_h, __ATOMIC_ACQUIRE) >> 32) != k)
            __builtin_ia32_pause();
        const int64_t t1 = now_ns();
        if (k > 200) us.push_back((t1 - t0) / 1000.0);
    }
    __atomic_store_n((uint64_t*)req_h, (uint64_t)0xFFFFFFFFu << 32, __ATOMIC_RELEASE);
    _mm_sfence();
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    std::sort(us.begin(), us.end());
    printf("%-60s %5u B: median %5.2f us  p90 %5.2f  p99 %5.2f\n", name, len, us[us.size() / 2],
           us[us.size() * 9 / 10], us[us.size() * 99 / 100]);
    fflush(stdout);
}

int main(int argc, char** argv) {
    const uint32_t len = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
    uint8_t *hreq = nullptr, *hreq_d = nullptr, *hack = nullptr, *hack_d = nullptr;
    if (hipHostMalloc((void**)&hreq, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostGetDevicePointer((void**)&hreq_d, hreq, 0) ||
        hipHostMalloc((void**)&hack, 4096, hipHostMallocMapped | hipHostMallocCoherent) ||
        hipHostGetDevicePointer((void**)&hack_d, hack, 0)) {
        fprintf(stderr, "host alloc failed\n");
        return 1;
    }
    run("request in pinned host memory (the product's block)", hreq, hreq_d, hack, hack_d, len);
    const struct { const char* name; unsigned flags; } kinds[] = {
        {"request in fine-grained device memory, host writes mapped", hipDeviceMallocFinegrained},
        {"request in uncached device memory, host writes mapped", hipDeviceMallocUncached},
    };
    for (const auto& kd : kinds) {
        uint8_t* d = nullptr;
        if (hipExtMallocWithFlags((void**)&d, 1 << 20, kd.flags) != hipSuccess) {
            (void)hipGetLastError();
            printf("%s: allocation refused\n", kd.name);
            continue;
        }
        hipPointerAttribute_t a;
        memset(&a, 0, sizeof a);
        (void)hipPointerGetAttributes(&a, d);
        printf("  %s: type %d, devicePointer %p, hostPointer %p\n", kd.name, (int)a.type,
               a.devicePointer, a.hostPointer);
        uint8_t* hv = a.hostPointer ? (uint8_t*)a.hostPointer : d;
        struct sigaction sa, old;
        memset(&sa, 0, sizeof sa);
        sa.sa_handler = on_segv;
        sigaction(SIGSEGV, &sa, &old);
        bool ok = false;
        if (sigsetjmp(jb, 1) == 0) {
            volatile uint64_t* p = (volatile uint64_t*)hv;
            *p = 0x1122334455667788ull;
            ok = *p == 0x1122334455667788ull;
        }
        sigaction(SIGSEGV, &old, nullptr);
        if (!ok) {
            printf("  %s: the host cannot write it through the pointer\n", kd.name);
            (void)hipFree(d);
            continue;
        }
        run(kd.name, hv, d, hack, hack_d, len);
        (void)hipFree(d);
    }
    return 0;
}
