// membw.hip — known-good HBM read ceiling on this box (guide §5.4 rule 10):
// every byte of a buffer read once with coalesced 16-B loads (plain and
// nontemporal), grid-stride, one u32 result per block so nothing is DCE'd.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <bool NT>
__global__ void __launch_bounds__(256) read_sum(const uint4* __restrict__ p, uint64_t n16,
                                                uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
#pragma unroll 4
    for (; i < n16; i += stride) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4* q = (const u32x4*)(p + i);
        u32x4 v = NT ? __builtin_nontemporal_load(q) : *q;
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    __shared__ uint32_t s[256];
    s[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0;
        for (int k = 0; k < 256; ++k) a += s[k];
        out[blockIdx.x] = a;
    }
}

extern "C" int membw_read(const void* p, uint64_t bytes, uint32_t* out, int blocks, int nt,
                          void* stream) {
    uint64_t n16 = bytes / 16;
    if (nt) hipLaunchKernelGGL(read_sum<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                               (const uint4*)p, n16, out);
    else hipLaunchKernelGGL(read_sum<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                            (const uint4*)p, n16, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Region pattern (the parse kernel's): each wave streams its own contiguous
// region in 1 KiB wave-wide loads, G loads per round trip (static count),
// 4 waves per workgroup, one wave per region.
template <int G>
__global__ void __launch_bounds__(256) read_region(const uint8_t* __restrict__ p, uint64_t region,
                                                   uint64_t nreg, uint32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint64_t w = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nreg) return;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const uint8_t* base = p + w * region;
    const uint64_t items = region / 1024;
    uint32_t acc = 0;
    for (uint64_t i = 0; i < items; i += G) {
        u32x4 v[G];
#pragma unroll
        for (int q = 0; q < G; ++q) {
            const uint64_t it = i + q < items ? i + q : items - 1;
            v[q] = __builtin_nontemporal_load(
                (const __attribute__((address_space(1))) u32x4*)(base + it * 1024 + lane * 16));
        }
#pragma unroll
        for (int q = 0; q < G; ++q) acc += v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    }
    out[w * 64 + lane] = acc;
}

extern "C" int membw_region(const void* p, uint64_t bytes, uint32_t* out, uint64_t region, int g,
                            void* stream) {
    const uint64_t nreg = bytes / region;
    const unsigned blocks = (unsigned)((nreg + 3) / 4);
    switch (g) {
    case 4: hipLaunchKernelGGL(read_region<4>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                               (const uint8_t*)p, region, nreg, out); break;
    case 8: hipLaunchKernelGGL(read_region<8>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                               (const uint8_t*)p, region, nreg, out); break;
    case 16: hipLaunchKernelGGL(read_region<16>, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                                (const uint8_t*)p, region, nreg, out); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Variants of the region pattern (A/B for the parse kernel's decomposition):
//   WAVES waves per workgroup; ILV = 1: wave w owns region w (as above);
//   ILV = 1 with WAVES = 1: the parse kernel's one-wave workgroups;
//   ILV = W: the W waves of a workgroup share W consecutive regions and
//   interleave their 1 KiB items (wave w reads items q*W + w), so the
//   resident waves read a denser band of memory.
template <int G, int WAVES, bool ILV>
__global__ void __launch_bounds__(64 * WAVES) read_region2(const uint8_t* __restrict__ p,
                                                           uint64_t region, uint64_t nreg,
                                                           uint32_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    uint64_t items, first, stride;
    const uint8_t* base;
    if (ILV) {
        const uint64_t g0 = (uint64_t)blockIdx.x * WAVES;       // first region of the block
        if (g0 >= nreg) return;
        const uint64_t nr = nreg - g0 < WAVES ? nreg - g0 : WAVES;
        base = p + g0 * region;
        items = nr * region / 1024;
        first = wid;
        stride = WAVES;
    } else {
        const uint64_t w = (uint64_t)blockIdx.x * WAVES + wid;
        if (w >= nreg) return;
        base = p + w * region;
        items = region / 1024;
        first = 0;
        stride = 1;
    }
    uint32_t acc = 0;
    for (uint64_t i = first; i < items; i += G * stride) {
        u32x4 v[G];
#pragma unroll
        for (int q = 0; q < G; ++q) {
            uint64_t it = i + q * stride;
            it = it < items ? it : items - 1;
            v[q] = __builtin_nontemporal_load(
                (const __attribute__((address_space(1))) u32x4*)(base + it * 1024 + lane * 16));
        }
#pragma unroll
        for (int q = 0; q < G; ++q) acc += v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    }
    out[((uint64_t)blockIdx.x * WAVES + wid) * 64 + lane] = acc;
}

extern "C" int membw_region2(const void* p, uint64_t bytes, uint32_t* out, uint64_t region,
                             int mode, void* stream) {
    const uint64_t nreg = bytes / region;
    hipStream_t s = (hipStream_t)stream;
    const uint8_t* q = (const uint8_t*)p;
    switch (mode) {
    case 0: hipLaunchKernelGGL((read_region2<8, 1, false>), dim3((unsigned)nreg), dim3(64), 0, s,
                               q, region, nreg, out); break;
    case 1: hipLaunchKernelGGL((read_region2<8, 4, false>), dim3((unsigned)((nreg + 3) / 4)),
                               dim3(256), 0, s, q, region, nreg, out); break;
    case 2: hipLaunchKernelGGL((read_region2<8, 4, true>), dim3((unsigned)((nreg + 3) / 4)),
                               dim3(256), 0, s, q, region, nreg, out); break;
    case 3: hipLaunchKernelGGL((read_region2<8, 8, true>), dim3((unsigned)((nreg + 7) / 8)),
                               dim3(512), 0, s, q, region, nreg, out); break;
    case 4: hipLaunchKernelGGL((read_region2<4, 8, true>), dim3((unsigned)((nreg + 7) / 8)),
                               dim3(512), 0, s, q, region, nreg, out); break;
    case 5: hipLaunchKernelGGL((read_region2<16, 1, false>), dim3((unsigned)nreg), dim3(64), 0, s,
                               q, region, nreg, out); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

typedef unsigned wg_u32x4 __attribute__((ext_vector_type(4)));

// Write granularity probe: 2^lg16 16-B stores per 128-B line, starting at
// chunk off16 of the line, over `lines` lines (grid-stride, coalesced).
template <bool NT>
__global__ void __launch_bounds__(256) write_gran(uint8_t* __restrict__ p, uint64_t lines,
                                                  int lg16, int off16, uint32_t v) {
    const uint64_t total = lines << lg16;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += stride) {
        const uint64_t line = t >> lg16;
        const uint32_t c = (uint32_t)(t & ((1u << lg16) - 1)) + off16;
        wg_u32x4* q = (wg_u32x4*)(p + line * 128 + c * 16);
        const wg_u32x4 x = {v, (uint32_t)t, (uint32_t)line, c};
        if (NT) __builtin_nontemporal_store(x, q);
        else *q = x;
    }
}

extern "C" int membw_write(void* p, uint64_t lines, int lg16, int off16, int nt, int blocks,
                           void* stream) {
    if (lg16 < 0 || lg16 > 3 || off16 < 0 || off16 + (1 << lg16) > 8) return -1;
    hipStream_t s = (hipStream_t)stream;
    if (nt)
        hipLaunchKernelGGL(write_gran<true>, dim3(blocks), dim3(256), 0, s, (uint8_t*)p, lines,
                           lg16, off16, 7u);
    else
        hipLaunchKernelGGL(write_gran<false>, dim3(blocks), dim3(256), 0, s, (uint8_t*)p, lines,
                           lg16, off16, 7u);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The parse kernel's access pattern without its work: one 64-lane workgroup
// per region (a tile), 1 KiB nontemporal wave loads in groups of 8, the
// parse kernel's LDS footprint per workgroup (so the same 18 waves fit a CU),
// and, with REC, one 16-B nontemporal store per lane at the end (the tile's
// records, 1 KiB per wave). Regions need not be multiples of 1 KiB: the last
// item re-reads inside the region, like the stream's clamped items.
template <bool REC>
__global__ void __launch_bounds__(64) read_tiles(const uint8_t* __restrict__ p, uint64_t region,
                                                 uint64_t nreg, uint32_t* __restrict__ out,
                                                 uint32_t lds_bytes) {
    extern __shared__ uint32_t lds[];
    const int lane = threadIdx.x;
    const uint64_t w = blockIdx.x;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const uint8_t* base = p + w * region;
    const uint64_t nch = region / 16, items = (nch + 63) / 64;
    uint32_t acc = 0;
    for (uint64_t i = 0; i < items; i += 8) {
        u32x4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            uint64_t c = (i + q) * 64 + lane;
            c = c < nch ? c : nch - 1;
            v[q] = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)(base + c * 16));
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    }
    lds[lane] = acc;                                   // the LDS is really allocated
    __builtin_amdgcn_wave_barrier();
    acc += lds[(lane + 1) & 63] + lds_bytes;
    if (REC && lds_bytes & 1) {                        // 8-B records (lds_bytes odd)
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        u32x2 r = {acc, acc};
        __builtin_nontemporal_store(r, (u32x2*)(out + (w * 64 + lane) * 2));
    } else if (REC) {
        u32x4 r = {acc, acc, acc, acc};
        __builtin_nontemporal_store(r, (u32x4*)(out + (w * 64 + lane) * 4));
    } else if (acc == 0x12345678u) {
        out[w * 64 + lane] = acc;
    }
}

extern "C" int membw_tiles(const void* p, uint64_t bytes, uint32_t* out, uint64_t region,
                           int rec, uint32_t lds_bytes, void* stream) {
    const uint64_t nreg = bytes / region;
    hipStream_t s = (hipStream_t)stream;
    if (rec) hipLaunchKernelGGL(read_tiles<true>, dim3((unsigned)nreg), dim3(64), lds_bytes, s,
                                (const uint8_t*)p, region, nreg, out, lds_bytes);
    else hipLaunchKernelGGL(read_tiles<false>, dim3((unsigned)nreg), dim3(64), lds_bytes, s,
                            (const uint8_t*)p, region, nreg, out, lds_bytes);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Copy pattern of the builder's payload pass: one wave per tile-sized region,
// 1 KiB nontemporal loads in groups of 8 from src, the same bytes stored to
// dst with plain 16-B stores (whole lines; no LDS).
__global__ void __launch_bounds__(64) copy_tiles(const uint8_t* __restrict__ src,
                                                 uint8_t* __restrict__ dst, uint64_t region) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x;
    const uint64_t w = blockIdx.x;
    const uint64_t nch = region / 16, items = (nch + 63) / 64;
    for (uint64_t i = 0; i < items; i += 8) {
        u32x4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            uint64_t c = (i + q) * 64 + lane;
            c = c < nch ? c : nch - 1;
            v[q] = __builtin_nontemporal_load(
                (const __attribute__((address_space(1))) u32x4*)(src + w * region + c * 16));
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint64_t c = (i + q) * 64 + lane;
            if (c < nch) *(u32x4*)(dst + w * region + c * 16) = v[q];
        }
    }
}

extern "C" int membw_copy_tiles(const void* src, void* dst, uint64_t bytes, uint64_t region,
                                void* stream) {
    const uint64_t nreg = bytes / region;
    hipLaunchKernelGGL(copy_tiles, dim3((unsigned)nreg), dim3(64), 0, (hipStream_t)stream,
                       (const uint8_t*)src, (uint8_t*)dst, region);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// FETCH_SIZE calibration by access width (the builder's dword
// blob loads were never calibrated). Every byte of the buffer read exactly
// once, coalesced, grid-stride, W bytes per lane per load (W = 4, 8, 16);
// STRIDE5: the builder's blob pattern (each lane 5 aligned dwords from its
// own 16-B chunk, adjacent lanes adjacent chunks: every byte read by one or
// two lanes, every line once from HBM).
template <int W>
__global__ void __launch_bounds__(256) read_width(const uint8_t* __restrict__ p, uint64_t n,
                                                  uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n / W; i += stride) {
        if constexpr (W == 1) {
            acc += p[i];
        } else if constexpr (W == 2) {
            acc += ((const uint16_t*)p)[i];
        } else if constexpr (W == 4) {
            acc += __builtin_nontemporal_load((const uint32_t*)p + i);
        } else if constexpr (W == 8) {
            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
            const u32x2 v = __builtin_nontemporal_load((const u32x2*)p + i);
            acc += v.x ^ v.y;
        } else {
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const u32x4 v = __builtin_nontemporal_load((const u32x4*)p + i);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(256) read_stride5(const uint8_t* __restrict__ p, uint64_t n,
                                                    uint32_t* __restrict__ out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    const uint32_t* d = (const uint32_t*)p;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i + 1 < n / 16; i += stride) {
        uint32_t v[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) v[k] = d[4 * i + k];
        acc += __builtin_amdgcn_alignbyte(v[1], v[0], 1) ^ v[2] ^ v[3] ^ v[4];
    }
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;
}

extern "C" int membw_width(const void* p, uint64_t bytes, uint32_t* out, int width, int blocks,
                           void* stream) {
    const uint8_t* q = (const uint8_t*)p;
    hipStream_t s = (hipStream_t)stream;
    if (width == 1) hipLaunchKernelGGL(read_width<1>, dim3(blocks), dim3(256), 0, s, q, bytes, out);
    else if (width == 2) hipLaunchKernelGGL(read_width<2>, dim3(blocks), dim3(256), 0, s, q, bytes, out);
    else if (width == 4) hipLaunchKernelGGL(read_width<4>, dim3(blocks), dim3(256), 0, s, q, bytes, out);
    else if (width == 8) hipLaunchKernelGGL(read_width<8>, dim3(blocks), dim3(256), 0, s, q, bytes, out);
    else if (width == 16) hipLaunchKernelGGL(read_width<16>, dim3(blocks), dim3(256), 0, s, q, bytes, out);
    else if (width == 5) hipLaunchKernelGGL(read_stride5, dim3(blocks), dim3(256), 0, s, q, bytes, out);
    else return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Write-allocate probe (round 4, the builder's read multiple): a 16-B-chunk
// copy src -> dst where every 128-B destination line gets only bytes
// [gap, 128) (gap = 0: whole lines). If FETCH_SIZE grows with gap > 0, partial
// line writes make the L2 fetch the rest of the line from HBM.
__global__ void __launch_bounds__(256) copy_gap(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                uint64_t n16, uint32_t gap16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        if ((uint32_t)(i & 7) < gap16) continue;          // 8 chunks per 128-B line
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)src + i);
        ((u32x4*)dst)[i] = v;
    }
}

extern "C" int membw_copy_gap(const void* src, void* dst, uint64_t bytes, int gap16, int blocks,
                              void* stream) {
    hipLaunchKernelGGL(copy_gap, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                       (const uint4*)src, (uint4*)dst, bytes / 16, (uint32_t)gap16);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// The in-place builder's access pattern without its work:
// read_tiles' stream over a tile of 64 frames of region/64 bytes each, then
// every lane writes back the whole 64-B sectors covering bytes [f, f + hdr)
// of its frame (f = its frame start: region/64 * lane, not 16-aligned), as
// the builder's header write-back does. policy: 0 plain stores, 1
// nontemporal, 2 write-through (sc1, system-coherent scope bit), 3 no write,
// 4 plain stores by the whole wave (frame-major, coalesced), 5 plain stores
// without the read, 6 / 7 = 0 / 4 after a ~12 us pause between the read and
// the write-back (the builder's chains run there: are the tile's lines still
// in L2 when its header sectors are written?).
// 8: each lane writes its sectors right after the group of loads holding its
// frame's start, 9: after the group holding its frame's end (a builder that
// writes a frame back as the stream passes it: the DRAM rows just read).
template <int POLICY>
__global__ void __launch_bounds__(64) hdr_tiles(uint8_t* __restrict__ p, uint64_t region,
                                                uint32_t hdr, uint32_t lds_bytes) {
    extern __shared__ uint32_t lds[];
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x;
    const uint64_t w = blockIdx.x;
    uint8_t* base = p + w * region;
    const uint64_t nch = region / 16, items = (nch + 63) / 64;
    uint32_t acc = 0;
    for (uint64_t i = 0; i < (POLICY == 5 ? 0 : items); i += 8) {
        u32x4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            uint64_t c = (i + q) * 64 + lane;
            c = c < nch ? c : nch - 1;
            v[q] = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)(base + c * 16));
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
        if (POLICY == 8 || POLICY == 9) {
            const uint64_t g0 = i * 1024, g1 = g0 + 8 * 1024;
            const uint64_t f = (uint64_t)lane * (region / 64);
            const uint64_t at = POLICY == 8 ? f : f + region / 64 - 1;
            if (at >= g0 && at < g1) {
                const u32x4 val = {acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
                const uint64_t s0 = f & ~63ull, s1 = (f + hdr + 63) & ~63ull;
                for (uint64_t a = s0; a < s1 && a + 16 <= region; a += 16)
                    *(__attribute__((address_space(1))) u32x4*)(base + a) = val;
            }
        }
    }
    if (POLICY == 8 || POLICY == 9) return;
    lds[lane] = acc;
    __builtin_amdgcn_wave_barrier();
    acc += lds[(lane + 1) & 63] + lds_bytes;
    if (POLICY >= 6) {
        for (int k = 0; k < 3; ++k) __builtin_amdgcn_s_sleep(127);
    }
    if (POLICY == 3) {
        if (acc == 0x12345678u) base[0] = 1;
        return;
    }
    u32x4 val = {acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
    if (POLICY == 4 || POLICY == 7) {
        // wave-cooperative: the 64 frames' sector ranges as one linear list of
        // 16-B chunks, consecutive lanes on consecutive chunks of a frame
        const uint32_t cmax = ((hdr + 63) / 64 + 1) * 4;
        for (uint32_t q = lane; q < 64 * cmax; q += 64) {
            const uint64_t j = q / cmax, k = q % cmax;
            const uint64_t fj = j * (region / 64);
            const uint64_t a = (fj & ~63ull) + 16 * k, e = (fj + hdr + 63) & ~63ull;
            if (a < e && a + 16 <= region)
                *(__attribute__((address_space(1))) u32x4*)(base + a) = val;
        }
        return;
    }
    const uint64_t f = (uint64_t)lane * (region / 64);
    const uint64_t s0 = f & ~63ull, s1 = (f + hdr + 63) & ~63ull;
    for (uint64_t a = s0; a < s1 && a + 16 <= region; a += 16) {
        __attribute__((address_space(1))) u32x4* q = (__attribute__((address_space(1))) u32x4*)(base + a);
        if (POLICY == 0 || POLICY == 5 || POLICY == 6) *q = val;
        else if (POLICY == 1) __builtin_nontemporal_store(val, q);
        else __hip_atomic_store((__attribute__((address_space(1))) uint64_t*)q, ((uint64_t)val.y << 32) | val.x,
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
             __hip_atomic_store((__attribute__((address_space(1))) uint64_t*)q + 1, ((uint64_t)val.w << 32) | val.z,
                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// The same header write-back in two phases (a builder that keeps its reads
// and its scattered writes apart in time): kernel 1 reads the tiles and
// writes each frame's 64-B header slot to a contiguous temp buffer; kernel 2
// reads the temp buffer and writes the whole 64-B sectors covering each
// frame's first `hdr` bytes (plain stores).
__global__ void __launch_bounds__(64) hdr_phase1(const uint8_t* __restrict__ p, uint64_t region,
                                                 uint8_t* __restrict__ tmp) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x;
    const uint64_t w = blockIdx.x;
    const uint8_t* base = p + w * region;
    const uint64_t nch = region / 16, items = (nch + 63) / 64;
    uint32_t acc = 0;
    for (uint64_t i = 0; i < items; i += 8) {
        u32x4 v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            uint64_t c = (i + q) * 64 + lane;
            c = c < nch ? c : nch - 1;
            v[q] = __builtin_nontemporal_load((const __attribute__((address_space(1))) u32x4*)(base + c * 16));
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) acc += v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
    }
    u32x4 val = {acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
    __attribute__((address_space(1))) u32x4* t = (__attribute__((address_space(1))) u32x4*)(tmp + w * 4096);
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k * 64 + lane] = val;          // 4 KiB per tile, coalesced
}
__global__ void __launch_bounds__(64) hdr_phase2(uint8_t* __restrict__ p, uint64_t region, uint32_t hdr,
                                                 const uint8_t* __restrict__ tmp) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const int lane = threadIdx.x;
    const uint64_t w = blockIdx.x;
    uint8_t* base = p + w * region;
    const __attribute__((address_space(1))) u32x4* t = (const __attribute__((address_space(1))) u32x4*)(tmp + w * 4096);
    u32x4 val = t[lane] ^ t[64 + lane] ^ t[128 + lane] ^ t[192 + lane];
    const uint64_t f = (uint64_t)lane * (region / 64);
    const uint64_t s0 = f & ~63ull, s1 = (f + hdr + 63) & ~63ull;
    for (uint64_t a = s0; a < s1 && a + 16 <= region; a += 16)
        *(__attribute__((address_space(1))) u32x4*)(base + a) = val;
}
extern "C" int membw_hdr_twophase(void* p, uint64_t bytes, uint64_t region, uint32_t hdr, void* tmp,
                                  int phases, void* stream) {
    const uint64_t nreg = bytes / region;
    hipStream_t s = (hipStream_t)stream;
    if (phases & 1) hipLaunchKernelGGL(hdr_phase1, dim3((unsigned)nreg), dim3(64), 0, s, (const uint8_t*)p, region, (uint8_t*)tmp);
    if (phases & 2) hipLaunchKernelGGL(hdr_phase2, dim3((unsigned)nreg), dim3(64), 0, s, (uint8_t*)p, region, hdr, (const uint8_t*)tmp);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int membw_hdr_tiles(void* p, uint64_t bytes, uint64_t region, uint32_t hdr, int policy,
                               uint32_t lds_bytes, void* stream) {
    const uint64_t nreg = bytes / region;
    hipStream_t s = (hipStream_t)stream;
    uint8_t* q = (uint8_t*)p;
    switch (policy) {
    case 0: hipLaunchKernelGGL(hdr_tiles<0>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 1: hipLaunchKernelGGL(hdr_tiles<1>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 2: hipLaunchKernelGGL(hdr_tiles<2>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 4: hipLaunchKernelGGL(hdr_tiles<4>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 5: hipLaunchKernelGGL(hdr_tiles<5>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 6: hipLaunchKernelGGL(hdr_tiles<6>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 7: hipLaunchKernelGGL(hdr_tiles<7>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 8: hipLaunchKernelGGL(hdr_tiles<8>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    case 9: hipLaunchKernelGGL(hdr_tiles<9>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    default: hipLaunchKernelGGL(hdr_tiles<3>, dim3((unsigned)nreg), dim3(64), lds_bytes, s, q, region, hdr, lds_bytes); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Device buffers of a chosen allocation kind (record-store cost by the
// records' memory type): 0 hipMalloc, 1 fine-grained, 2 uncached,
// 3 contiguous. Returns NULL on failure.
extern "C" void* membw_alloc(uint64_t bytes, int kind) {
    void* p = nullptr;
    hipError_t e;
    switch (kind) {
    case 0: e = hipMalloc(&p, bytes); break;
    case 1: e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained); break;
    case 2: e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached); break;
    default: e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous); break;
    }
    return e == hipSuccess ? p : nullptr;
}
extern "C" void membw_free(void* p) { (void)hipFree(p); }
