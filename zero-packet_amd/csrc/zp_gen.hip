// zp_gen.hip — device-side synthetic batch generator (a batched
// PacketBuilder restricted to the frame shapes of BASELINE.json configs 1-5;
// the reference builder is builder.rs:94-909). Byte content is defined once
// in zp_gen.h; this file only maps it onto the GPU:
//   zp_gen_lengths_kernel: thread per packet, plan -> frame length.
//   zp_gen_frames_kernel:  wave per packet. Lanes produce 16-B arena-aligned
//     chunks of the frame, sum the L4 segment (wave reduction) to fill the
//     checksum, then store interior chunks as dwordx4 and the (at most two)
//     partial edge chunks bytewise, so neighbouring frames never race.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/zero_packet.h"
#include "zp_gen.h"

__global__ void zp_gen_lengths_kernel(int cfg, uint64_t seed, uint64_t first, uint64_t n,
                                      uint32_t* lens) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    zp_plan p;
    zp_plan_packet(cfg, seed, first + i, &p);
    lens[i] = p.len;
}

// Bytes [pos, pos + 16) of the frame as two little-endian u64 (positions
// outside [0, len) are 0).
struct Chunk16 { uint64_t lo, hi; };

__device__ Chunk16 gen_chunk16(const zp_plan* p, int64_t pos) {
    Chunk16 c = {0, 0};
    uint64_t word = 0;
    int64_t wi = -1;
    for (int j = 0; j < 16; ++j) {
        int64_t x = pos + j;
        uint64_t b = 0;
        if (x >= 0 && x < (int64_t)p->len) {
            if (x >= p->pay_off) {
                int64_t q = x - p->pay_off;
                if ((q >> 3) != wi) { wi = q >> 3; word = zp_h(p->key, ZP_S_PAY + 64u * (uint64_t)wi); }
                b = (word >> (8 * (q & 7))) & 0xFF;
            } else {
                b = zp_gen_byte(p, (uint32_t)x);
            }
        }
        if (j < 8) c.lo |= b << (8 * j);
        else c.hi |= b << (8 * (j - 8));
    }
    return c;
}

__device__ __forceinline__ uint32_t chunk_byte(const Chunk16& c, int j) {
    return (uint32_t)(((j < 8) ? (c.lo >> (8 * j)) : (c.hi >> (8 * (j - 8)))) & 0xFF);
}

__global__ void __launch_bounds__(256)
zp_gen_frames_kernel(int cfg, uint64_t seed, uint64_t first, uint64_t n,
                     uint8_t* arena, const uint64_t* offs) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t i = wave; i < n; i += nwaves) {
        zp_plan p;
        zp_plan_packet(cfg, seed, first + i, &p);
        zp_plan_ip_csums(&p);
        // L4 segment sum in reference word parity (words start at l4_off).
        uint32_t s = 0;
        for (uint32_t x = p.l4_off + 16u * lane; x < p.len; x += 1024u) {
            Chunk16 c = gen_chunk16(&p, x);
            // Big-endian word sum: even j is the high byte (x - l4_off is even).
            uint64_t ev = 0, od = 0;
            ev = (c.lo & 0x00FF00FF00FF00FFull) + (c.hi & 0x00FF00FF00FF00FFull);
            od = ((c.lo >> 8) & 0x00FF00FF00FF00FFull) + ((c.hi >> 8) & 0x00FF00FF00FF00FFull);
            uint32_t e = 0, o = 0;
            for (int k = 0; k < 4; ++k) { e += (ev >> (16 * k)) & 0xFFFF; o += (od >> (16 * k)) & 0xFFFF; }
            s += (e << 8) + o;
        }
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) s += __shfl_xor(s, d, 64);
        p.csum_l4 = zp_plan_l4_csum(&p, s);
        // Store.
        uint8_t* f = arena + offs[i];
        uintptr_t fa = (uintptr_t)f;
        uintptr_t base = fa & ~(uintptr_t)15;
        uintptr_t end = fa + p.len;
        for (uintptr_t c = base + 16u * lane; c < end; c += 1024u) {
            int64_t pos = (int64_t)(c - fa);
            Chunk16 b = gen_chunk16(&p, pos);
            if (c >= fa && c + 16 <= end) {
                uint4 v;
                v.x = (uint32_t)b.lo; v.y = (uint32_t)(b.lo >> 32);
                v.z = (uint32_t)b.hi; v.w = (uint32_t)(b.hi >> 32);
                *(uint4*)c = v;
            } else {
                for (int j = 0; j < 16; ++j) {
                    uintptr_t a = c + j;
                    if (a >= fa && a < end) *(uint8_t*)a = (uint8_t)chunk_byte(b, j);
                }
            }
        }
    }
}

extern "C" int zp_gen_lengths_device(int config, uint64_t seed, uint64_t first, uint64_t n,
                                     uint32_t* lens, void* stream) {
    if (n == 0) return 0;
    if (config < 1 || config > 6 || !lens) return -1;
    uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(zp_gen_lengths_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, config, seed, first, n, lens);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int zp_gen_frames_device(int config, uint64_t seed, uint64_t first, uint64_t n,
                                    uint8_t* arena, const uint64_t* offs,
                                    const uint32_t* lens, void* stream) {
    (void)lens;
    if (n == 0) return 0;
    if (config < 1 || config > 6 || !arena || !offs) return -1;
    uint64_t waves = n < (1ull << 20) ? n : (1ull << 20);
    uint64_t blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(zp_gen_frames_kernel, dim3((unsigned)blocks), dim3(256), 0,
                       (hipStream_t)stream, config, seed, first, n, arena, offs);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
