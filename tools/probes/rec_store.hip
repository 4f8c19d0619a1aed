// Record-store probe (lab tool, not product): the parse's tile pattern
// (zp_probe_tiles_device, zp_stats.hip) with its 8-B record stores issued in
// other ways, to see which costs less inside the read stream.
//   mode 0  no stores
//   1  64 lanes x 8 B nontemporal at the tile's end (the parse's way)
//   2  the same, default cache policy
//   3  nontemporal, before the tile's loads (the stores' time in the wave)
//   4  32 lanes x 16 B nontemporal at the end (same bytes, half the lanes)
//   5  nontemporal into a 2 MiB ring (L2-resident: the cost without HBM)
//   6  nontemporal after half of the tile's loads
//   7  nontemporal into the arena slice just read (row locality; scratch arena)
//   8  default policy into the 2 MiB ring (stays in L2: no memory writes)
//   9  the same bytes as 1 in two 4-B store instructions
//  10  1 plus a second 64 x 8 B nontemporal store into the ring (two stores)
//  11-14  2 / 4 / 8 / 16 nontemporal 64 x 8 B store instructions per tile into
//      consecutive 512-B blocks of a buffer of 16 blocks per tile (`wide`)
//  15 / 16  the same bytes as 1 in bigger bursts: every 4th / 16th tile's wave
//      stores the records of 4 / 16 tiles (2 / 8 KiB), the others none
//  17 / 18  64 lanes x 4 B / 2 B nontemporal at the end (a 4-B / 2-B record:
//      does the cost follow the bytes?)
//  19  the low 4 B of each 8-B record only (stride 8: the same lines, half
//      the bytes); 20: 19, plus the high 4 B for every 4th lane
//  21  a 64-B compressed tile slot (16 lanes x 4 B) at the start of the
//      tile's record block; 22: the same slot as 4 lanes x 16 B
// and per run: k consecutive tiles per wave, LDS bytes per wave (8960: the
// parse's 18 waves per CU; 7680: 21; 4096: the VGPR bound)
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
#define G __attribute__((address_space(1)))

template <int LDSB>
__global__ void __launch_bounds__(64) rec_probe_kernel(const uint8_t* __restrict__ p, uint64_t nchunks,
                                                       uint64_t cpt, uint64_t n,
                                                       const uint64_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ lens,
                                                       uint64_t* __restrict__ rec,
                                                       uint64_t* __restrict__ ring,
                                                       uint64_t* __restrict__ wide, int mode, int k,
                                                       uint32_t* __restrict__ sink) {
    __shared__ uint32_t pad[LDSB / 4];
    const uint32_t lane = threadIdx.x;
    const G u32x4* q = (const G u32x4*)p;
    for (int j = 0; j < k; ++j) {
    const uint64_t t = (uint64_t)blockIdx.x * k + j;
    if (64 * t >= n) return;
    const uint64_t c0 = t * cpt;
    const uint64_t c1 = (t + 1) * cpt < nchunks ? (t + 1) * cpt : nchunks;
    const uint64_t i = 64 * t + lane < n ? 64 * t + lane : n - 1;
    uint32_t acc = (uint32_t)offs[i] ^ lens[i];
    const uint64_t word = ((uint64_t)lane << 32) | (uint32_t)t;
    if (mode == 3) __builtin_nontemporal_store(word, rec + 64 * t + lane);
    const uint64_t half = c0 + ((c1 - c0) / 2 & ~(uint64_t)63);
    uint64_t c = c0 + lane;
    for (; c + 192 < c1; c += 256) {
        const u32x4 a = __builtin_nontemporal_load(q + c);
        const u32x4 b = __builtin_nontemporal_load(q + c + 64);
        const u32x4 d = __builtin_nontemporal_load(q + c + 128);
        const u32x4 e = __builtin_nontemporal_load(q + c + 192);
        acc ^= (a.x ^ b.y) ^ (d.z ^ e.w);
        if (mode == 6 && c < half && c + 256 >= half)
            __builtin_nontemporal_store(word ^ acc, rec + 64 * t + lane);
    }
    for (; c < c1; c += 64) {
        const u32x4 a = __builtin_nontemporal_load(q + c);
        acc ^= a.x ^ a.w;
    }
    pad[lane] = acc;
    __builtin_amdgcn_wave_barrier();
    acc ^= pad[lane ^ 1];
    __builtin_amdgcn_wave_barrier();
    const uint64_t w = word ^ acc;
    if (mode == 1) __builtin_nontemporal_store(w, rec + 64 * t + lane);
    else if (mode == 2) rec[64 * t + lane] = w;
    else if (mode == 4) {
        if (lane < 32) __builtin_nontemporal_store(u64x2{w, w ^ 1}, (u64x2*)(rec + 64 * t) + lane);
    } else if (mode == 5) __builtin_nontemporal_store(w, ring + 64 * (t & 4095) + lane);
    else if (mode == 7) __builtin_nontemporal_store(w, (uint64_t*)(p + 16 * c0) + lane);
    else if (mode == 8) ring[64 * (t & 4095) + lane] = w;
    else if (mode == 15 || mode == 16) {
        const uint64_t g = mode == 15 ? 4 : 16;
        if (t % g == 0)
            for (uint64_t b = 0; b < g; ++b)
                if (64 * (t + b) + lane < n)
                    __builtin_nontemporal_store(w ^ b, rec + 64 * (t + b) + lane);
    } else if (mode >= 11 && mode <= 14) {
        const int m = 1 << (mode - 10);
        for (int b = 0; b < m; ++b)
            __builtin_nontemporal_store(w ^ (uint64_t)b, wide + (16 * t + b) * 64 + lane);
    }
    else if (mode == 17) __builtin_nontemporal_store((uint32_t)w, (uint32_t*)(rec + 64 * t) + lane);
    else if (mode == 18) __builtin_nontemporal_store((uint16_t)w, (uint16_t*)(rec + 64 * t) + lane);
    else if (mode == 21) {
        if (lane < 16) __builtin_nontemporal_store((uint32_t)w, (uint32_t*)(rec + 64 * t) + lane);
    } else if (mode == 22) {
        if (lane < 4) __builtin_nontemporal_store(u64x2{w, w ^ 3}, (u64x2*)(rec + 64 * t) + lane);
    }
    else if (mode == 19 || mode == 20) {
        __builtin_nontemporal_store((uint32_t)w, (uint32_t*)(rec + 64 * t + lane));
        if (mode == 20 && (lane & 3) == 0)
            __builtin_nontemporal_store((uint32_t)(w >> 32), (uint32_t*)(rec + 64 * t + lane) + 1);
    }
    else if (mode == 9) {
        __builtin_nontemporal_store((uint32_t)w, (uint32_t*)(rec + 64 * t) + lane);
        __builtin_nontemporal_store((uint32_t)(w >> 32), (uint32_t*)(rec + 64 * t) + 64 + lane);
    } else if (mode == 10) {
        __builtin_nontemporal_store(w, rec + 64 * t + lane);
        __builtin_nontemporal_store(w ^ 7, ring + 64 * (t & 4095) + lane);
    }
    else if (mode == 0 && acc == 0x9E3779B9u) sink[0] = acc;
    }
}

extern "C" int rec_probe(const uint8_t* p, uint64_t bytes, uint64_t n, const uint64_t* offs,
                         const uint32_t* lens, void* rec, void* ring, void* wide, int mode, int k,
                         int lds,
                         uint32_t* sink, void* stream) {
    const uint64_t tiles = (n + 63) / 64, nchunks = bytes / 16;
    const uint64_t cpt = (nchunks + tiles - 1) / tiles;
    const unsigned grid = (unsigned)((tiles + k - 1) / k);
    hipStream_t s = (hipStream_t)stream;
    if (lds == 8960)
        hipLaunchKernelGGL(rec_probe_kernel<8960>, dim3(grid), dim3(64), 0, s, p, nchunks, cpt, n,
                           offs, lens, (uint64_t*)rec, (uint64_t*)ring, (uint64_t*)wide, mode, k, sink);
    else if (lds == 7680)
        hipLaunchKernelGGL(rec_probe_kernel<7680>, dim3(grid), dim3(64), 0, s, p, nchunks, cpt, n,
                           offs, lens, (uint64_t*)rec, (uint64_t*)ring, (uint64_t*)wide, mode, k, sink);
    else
        hipLaunchKernelGGL(rec_probe_kernel<4096>, dim3(grid), dim3(64), 0, s, p, nchunks, cpt, n,
                           offs, lens, (uint64_t*)rec, (uint64_t*)ring, (uint64_t*)wide, mode, k, sink);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The expansion pass of a compressed-slot scheme: one wave per tile reads the
// tile's 64-B slot (lane l: dword l & 15) and writes the tile's 64 8-B records.
__global__ void __launch_bounds__(256) expand_probe_kernel(uint64_t* __restrict__ rec, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t t = i / 64;
    const uint32_t lane = threadIdx.x & 63;
    if (64 * t >= n) return;
    const uint32_t d = ((const uint32_t*)(rec + 64 * t))[lane & 15];
    const uint32_t m = __shfl(d, 0);
    const uint32_t ix = (__shfl(d, 10 + (lane >> 4)) >> (2 * (lane & 15))) & 3u;
    const uint32_t lo = __shfl(d, 2 + 2 * ix), hi = __shfl(d, 3 + 2 * ix);
    if (m == 0xFFFFFFFFu) return;                       // (never in the probe)
    if (i < n) __builtin_nontemporal_store(((uint64_t)hi << 32) | lo, rec + i);
}
extern "C" int expand_probe(void* rec, uint64_t n, void* stream) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(expand_probe_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (uint64_t*)rec, n);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
