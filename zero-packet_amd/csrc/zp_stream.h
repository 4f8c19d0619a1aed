// zp_stream.h — the packed stream of the batch kernels: every byte of a
// tile's 64 frames read once by full 1 KiB wave loads, with the per-frame word
// sums, header windows and last chunks staged in LDS.
// Shared by zp_parse.hip (PacketParser::parse) and zp_build.hip (the batched
// builder's lane-per-frame path).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef ZP_WIN
#define ZP_WIN 128           // LDS header window bytes per frame (multiple of 16)
#endif
#define ZP_WIN_CH (ZP_WIN / 16)
// The window cell index (chunk * 64 + rank) travels in 10 bits of the item
// descriptor (KEEP_WIN): at most 16 chunks.
static_assert(ZP_WIN % 16 == 0 && ZP_WIN <= 256, "ZP_WIN must be a multiple of 16, <= 256");
#define ZP_GIANT 65536u      // frames longer than this take the exact path
#define ZP_G 8               // stream items (1 KiB loads) per group

// All loads go through address_space(1) pointers: pointers rebuilt from
// integers would otherwise compile to FLAT loads, which count against both
// vmcnt and lgkmcnt, so every LDS wait would also drain in-flight HBM loads.
#define ZP_GLOBAL __attribute__((address_space(1)))
typedef unsigned zp_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned zp_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 ldg16(uintptr_t a) {
    zp_u32x4 v = *(const ZP_GLOBAL zp_u32x4*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t ldg4(uintptr_t a) { return *(const ZP_GLOBAL uint32_t*)a; }

// Streamed 16-B chunk, read once: nontemporal.
__device__ __forceinline__ uint4 ld_stream(uintptr_t a) {
    zp_u32x4 v = __builtin_nontemporal_load((const ZP_GLOBAL zp_u32x4*)a);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// System-scope 16-B load for frames in fine-grained host memory that the host
// rewrites while the kernel runs (zp_parse_one's resident server, whose block
// of ZP_SYS_BYTES starts at `base`): one buffer load with sc0 sc1 (system
// scope: past the vector L1 and the L2), so no cache-wide invalidate is
// needed after the doorbell. Addresses outside the block (the dummy loads of
// an empty tile) read 0 instead of faulting.
#define ZP_SYS_BYTES (128u + (64u << 10) + 64u)   // = zp_ctx.hip's mapped block
__device__ __forceinline__ uint4 ld_sys16(uintptr_t base, uintptr_t a) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)ZP_SYS_BYTES, 0x00020000);
    const zp_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(uint32_t)(a - base), 0,
                                                              1 | 16);   // sc0 sc1
    return make_uint4(v.x, v.y, v.z, v.w);
}
// ... and the matching stores (write-through to the host, no L2 write-back
// needed before the acknowledgement).
__device__ __forceinline__ void st_sys8(void* p, uint64_t v) {
    __hip_atomic_store((ZP_GLOBAL uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// One 16-B write-through vector store at a (16-B aligned, inside the block):
// a single write request, so the host sees its 16 bytes together.
__device__ __forceinline__ void st_sys16(uintptr_t base, uintptr_t a, zp_u32x4 v) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)ZP_SYS_BYTES, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(uint32_t)(a - base), 0, 1 | 16);   // sc0 sc1
}

// A readable 16-B chunk for masked lanes of frames that own no bytes.
static __device__ uint4 zp_safe_chunk;

// Keep bytes [lo, hi) of the dword whose first byte is at position `base`.
__device__ __forceinline__ uint32_t byte_mask(int base, int lo, int hi) {
    int a = lo - base, b = hi - base;
    a = a < 0 ? 0 : (a > 4 ? 4 : a);
    b = b < 0 ? 0 : (b > 4 ? 4 : b);
    uint64_t m = ((1ull << (8 * b)) - 1ull) & ~((1ull << (8 * a)) - 1ull);
    return (uint32_t)m;
}

// Little-endian 16-bit word sum of a dword: (x & 0xFFFF) + (x >> 16) + acc.
__device__ __forceinline__ uint32_t sad16(uint32_t x, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(x, 0u, acc);
}

// V-sum of bytes [l, h) of a 16-B chunk (0 <= l < h <= 16).
__device__ __forceinline__ uint32_t chunk_sum(uint4 v, int l, int h, uint32_t s) {
    if (l == 0 && h == 16) {
        s = sad16(v.x, s); s = sad16(v.y, s); s = sad16(v.z, s); s = sad16(v.w, s);
    } else {
        s = sad16(v.x & byte_mask(0, l, h), s);
        s = sad16(v.y & byte_mask(4, l, h), s);
        s = sad16(v.z & byte_mask(8, l, h), s);
        s = sad16(v.w & byte_mask(12, l, h), s);
    }
    return s;
}

// x != 0 && x == 0 (mod 65535) for a u32 x, by two end-around-carry folds
// (2^16 == 1 mod 65535; the second fold leaves 1..65535 for x != 0) instead of
// a 32-bit modulo (a multiply-high sequence).
__device__ __forceinline__ bool nz_mod65535_zero(uint32_t x) {
    const uint32_t y = (x & 0xFFFFu) + (x >> 16);
    return x != 0 && (y & 0xFFFFu) + (y >> 16) == 65535u;
}

// Checksum validity from the arena-parity sum V of a segment starting at an
// address of parity `odd`, with accumulator acc (fast path, exact V).
__device__ __forceinline__ bool csum_ok(uint32_t acc, uint32_t V, bool odd) {
    if (acc == 0 && V == 0) return false;                  // S == 0 -> 0xFFFF
    // 2^16 == 1 (mod 65535): t = acc + W folded by 16-bit limbs (t < 2^41);
    // t > 0 here, so t == 0 (mod 65535) iff the folds end at 65535 (the
    // modulo form below checked against it on 4M random and edge inputs;
    // c5 -0.8 %, c3/c4 +-0.1 %, profiles/r05_kbench_csum_fold.log)
    const uint64_t t = (uint64_t)acc + (odd ? (uint64_t)V : (uint64_t)V << 8);
    uint32_t x = (uint32_t)(t & 0xFFFFu) + (uint32_t)((t >> 16) & 0xFFFFu) + (uint32_t)(t >> 32);
    x = (x & 0xFFFFu) + (x >> 16);
    x = (x & 0xFFFFu) + (x >> 16);
    return x == 65535u;
}

// --------------------------------------------------------------------------
// Cross-lane scans (DPP).
// --------------------------------------------------------------------------

// Inclusive wave-wide prefix sum: row_shr 1/2/4/8 scan each 16-lane row,
// row_bcast 15/31 carry the row totals upward.
__device__ __forceinline__ uint32_t wave_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return __builtin_amdgcn_readlane(v, (int)l);
}

// V-sum of bytes [lo, hi) of a 16-B chunk (0 <= lo <= hi <= 16).
__device__ __forceinline__ uint32_t range_sum(uint4 v, uint32_t lo, uint32_t hi) {
    uint32_t s = 0;
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int a = (int)lo - 4 * i, b = (int)hi - 4 * i;
        const uint32_t na = a < 0 ? 0u : (a > 4 ? 4u : (uint32_t)a);
        const uint32_t nb = b < 0 ? 0u : (b > 4 ? 4u : (uint32_t)b);
        const uint32_t m = (uint32_t)(0xFFFFFFFFull >> (32u - 8u * nb)) &
                           ~(uint32_t)(0xFFFFFFFFull >> (32u - 8u * na));
        s = sad16(d[i] & m, s);
    }
    return s;
}

// --------------------------------------------------------------------------
// The stream. Every byte of a frame is read exactly once, by one wave-wide
// coalesced stream: the 16-B chunks [A & ~15, E) of the wave's frames are
// concatenated into one virtual sequence of T chunks (exclusive scan of the
// per-frame chunk counts) and read in items of 64 chunks, so every load
// instruction is a full 1 KiB whatever the frame lengths, and the chunks of
// a 128-B line shared by two neighbouring frames are read by adjacent lanes
// of the same or the next item (no second HBM fetch).
//
// Frames that own chunks are numbered by rank (compaction of the wave's
// non-empty frames). Lane l of item i reads virtual chunk vv = 64i + l of
// frame rank r(vv): a scalar loop sets one bit of a 64-bit mask F per frame
// starting inside the item, and r = (frames started before the item) - 1 +
// popcount(F & lanes <= l) is one v_mbcnt pair; the frame's address and
// bounds then come from its rank with ds_bpermute. Per-frame sums need no
// segmented reduction: with C(vv) the running inclusive sum of the stream,
// the lane holding a frame's last chunk records C there, and the frame's sum
// is C(last of r) - C(last of r - 1).
// The first 8 chunks of each frame (the header window) and its last chunk
// are also written to LDS for the walk and the verdict.
// --------------------------------------------------------------------------
struct Cursor {          // wave-uniform
    uint32_t rbase;      // rank of the frame holding the chunk before the item
    uint32_t nz;         // number of ranks (frames that own chunks)
    uint64_t* starts;    // LDS: starts[i % ZP_STARTS] = bit b set <=> a frame starts at 64i + b
};

struct Ranked {          // lane r = frame of rank r
    uint32_t org_lo, org_hi;   // (A & ~15) - 16 * pfx
    uint32_t last;       // last virtual chunk
    uint32_t pfx;        // first virtual chunk
    uint32_t mid;        // T4 streams: (virtual chunk << 4) | byte of a marked frame offset, or ~0
};

// Per-lane item descriptor.
#define KEEP_IN (1u << 31)     // chunk belongs to a frame (else past the end)
#define KEEP_WIN (1u << 30)    // chunk index < ZP_WIN_CH: window cell in bits 0-9
#define KEEP_TAIL (1u << 29)   // frame's last chunk
#define ZP_T4N 3               // chunks kept before each frame's last one (T4 streams, <= 3)
#define KEEP_T4 (1u << 28)     // one of the ZP_T4N chunks before the frame's last (T4 streams) ...
#define KEEP_T4D(k) (((k) >> 22) & 3u)   // ... at this distance from the last, minus 1
#define KEEP_MID (1u << 27)    // (T4 streams) the chunk of the frame's marked offset, its byte in 10-13
#define KEEP_MIDB(k) (((k) >> 10) & 15u)
#define KEEP_CELL(k) ((k) & 0x3FFu)
#define KEEP_RANK(k) (((k) >> 16) & 63u)

__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t r) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(r << 2), (int)v);
}

#define ZP_STARTS 64           // items per rebuild of the frame-start masks (a power of two >= ZP_G)
// Rebuilds the start masks of items [w0, w0 + ZP_STARTS): one LDS atomic OR per
// frame starting there. Straight-line code (no loop): a loop here would make
// LLVM's wait-count insertion drain the group in flight (vmcnt(0)).
__device__ __forceinline__ void build_starts(uint32_t w0, const Cursor& c, const Ranked& R,
                                             int lane) {
    if ((uint32_t)lane < (uint32_t)ZP_STARTS) c.starts[lane] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint32_t it = R.pfx >> 6;
    if ((uint32_t)lane < c.nz && it >= w0 && it < w0 + (uint32_t)ZP_STARTS)
        __hip_atomic_fetch_or(&c.starts[it - w0], 1ull << (R.pfx & 63u), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WAVEFRONT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Always issues exactly G loads (items past the end re-read the wave's last
// chunk, or a dummy): a static load count keeps the compiler's s_waitcnt
// exact.
template <int G, bool T4 = false>
__device__ __forceinline__ void issue_group(uint32_t i0, uint32_t nitems, Cursor& c,
                                            const Ranked& R, int lane, uintptr_t fallback,
                                            uint4 (&v)[G], uint32_t (&keep)[G]) {
    uintptr_t a[G];
    // The G items' frame-start masks in one LDS round trip (G divides 64, so
    // the group never straddles a rebuild of the mask table).
    static_assert(ZP_STARTS % G == 0 && G % 2 == 0 && ZP_STARTS <= 64,
                  "group size must be even and divide ZP_STARTS");
    if ((i0 & (ZP_STARTS - 1u)) == 0 && i0 < nitems) build_starts(i0, c, R, lane);   // wave-uniform
    // G/2 ds_read_b128 issued back to back, then one wait
    uint64_t Fq[G];
    zp_u32x4 m[G / 2];
    const zp_u32x4* sp = (const zp_u32x4*)&c.starts[i0 & (ZP_STARTS - 1u)];
#pragma unroll
    for (int q = 0; q < G / 2; ++q) m[q] = sp[q];
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const uint32_t lo = (q & 1) ? m[q / 2].z : m[q / 2].x;
        const uint32_t hi = (q & 1) ? m[q / 2].w : m[q / 2].y;
        // (readfirstlane returns int: cast before widening, no sign extension)
        const uint64_t fu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(hi) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane(lo);
        Fq[q] = i0 + q < nitems ? fu : 0ull;
    }
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const uint32_t i = i0 + q;
        const uint32_t base = 64u * i;
        const uint64_t F = Fq[q];
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(F >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)F, 0u));
        uint32_t r = c.rbase + below + (uint32_t)((F >> lane) & 1u);
        r = r < c.nz ? r : c.nz - 1u;       // past the last frame (and never a stray lane)
        c.rbase += (uint32_t)__builtin_popcountll(F);
        const uint32_t vv = base + (uint32_t)lane;
        const uint32_t olo = bperm(R.org_lo, r), ohi = bperm(R.org_hi, r);
        const uint32_t lv = bperm(R.last, r), fp = bperm(R.pfx, r);
        const uint32_t ci = vv - fp;                          // chunk index within the frame
        uint32_t k = (r & 63u) << 16;
        k |= ci < ZP_WIN_CH ? KEEP_WIN | (ci * 64u + ((r ^ ci) & 63u)) : 0u;
        k |= vv == lv ? KEEP_TAIL : 0u;
        if (T4) {
            k |= lv - vv - 1u < (uint32_t)ZP_T4N ? KEEP_T4 | ((lv - vv - 1u) << 22) : 0u;
            const uint32_t md = bperm(R.mid, r);
            k |= (md >> 4) == vv ? KEEP_MID | ((md & 15u) << 10) : 0u;
        }
        keep[q] = (i < nitems && vv <= lv) ? k | KEEP_IN : 0u;
        const uint32_t vc = vv < lv ? vv : lv;
        a[q] = nitems ? (((uintptr_t)ohi << 32) | olo) + 16ull * vc : fallback;
    }
#pragma unroll
    for (int q = 0; q < G; ++q) v[q] = ld_stream(a[q]);
    // Compiler barrier: keeps LLVM from sinking the loads below the consume
    // of the previous group (which would serialise the double buffer).
    asm volatile("" ::: "memory");
}

// An empty asm that reads every register of the group: forces the wait for
// all of its loads at this point.
template <int G>
__device__ __forceinline__ void retire_group(const uint4 (&v)[G]) {
#pragma unroll
    for (int q = 0; q < G; ++q) asm volatile("" ::"v"(v[q].x), "v"(v[q].y), "v"(v[q].z), "v"(v[q].w));
}

template <int G, bool T4 = false>
__device__ __forceinline__ void consume_group(uint32_t i0, uint32_t nitems, int lane,
                                              const uint4 (&v)[G], const uint32_t (&keep)[G],
                                              uint4* win, uint4* tail, uint32_t* cend,
                                              uint32_t& run, uint4* t4 = nullptr,
                                              uint32_t* cmid = nullptr) {
    // Items past the end (wave-uniform) are skipped by a branch, not a
    // loop exit: with `break` LLVM stops fully unrolling past G = 8 and the
    // group arrays go to scratch.
#pragma unroll
    for (int q = 0; q < G; ++q) {
        const uint32_t i = i0 + q;
        if (i >= nitems) continue;                            // wave-uniform
        const uint32_t k = keep[q];
        if (k & KEEP_WIN) win[KEEP_CELL(k)] = v[q];
        // T4 streams (the builder) also keep the 3 chunks before each
        // frame's last one: t4[rank * 3 + distance from the last - 1]
        if (T4 && (k & KEEP_T4)) t4[KEEP_RANK(k) * ZP_T4N + KEEP_T4D(k)] = v[q];
        uint32_t part = sad16(v[q].x, 0u);
        part = sad16(v[q].y, part);
        part = sad16(v[q].z, part);
        part = sad16(v[q].w, part);
        const uint32_t P = wave_scan(k & KEEP_IN ? part : 0u);
        if (k & KEEP_TAIL) {
            if (tail != nullptr) tail[KEEP_RANK(k)] = v[q];
            cend[KEEP_RANK(k)] = run + P;
        }
        // T4 streams: the running sum through the marked byte of a frame
        // (its chunks before it and the chunk's bytes before the mark)
        if (T4 && (k & KEEP_MID)) cmid[KEEP_RANK(k)] = run + P - part + range_sum(v[q], 0u, KEEP_MIDB(k));
        run += rdl(P, 63);
    }
    // Retire the dummy loads of a short last group here: a load still in
    // flight on some path makes the compiler wait vmcnt(0) at the next issue.
    retire_group(v);
}

// --------------------------------------------------------------------------
// The batch kernel.
// --------------------------------------------------------------------------
// One tile = 64 consecutive frames on one wave (lane = frame).
struct WaveLds {
    uint4 win[(ZP_WIN_CH + 1) * 64];   // header windows [ZP_WIN_CH][64] (+ last chunks [64])
    uint32_t cend[64];                      // running stream sum at each frame's last chunk
    uint64_t starts[ZP_STARTS];             // per-item frame-start masks
};

struct TileState {
    uint64_t tile;
    uintptr_t ga;            // this lane's frame
    uint32_t len, shift, wlen, rank;
    bool live, giant;
    uint32_t nitems;         // wave-uniform
    uint64_t ranked;         // wave-uniform: lanes whose frames own chunks (rank order = lane order)
    Ranked R;
    Cursor cur;
    uint32_t run;            // running stream sum
};

// Chunk ranges, ranks and the compacted per-rank frame table of a tile.
// len = 0 lanes (past the batch) own no chunks.
template <class L>
__device__ __forceinline__ void tile_setup(TileState& s, uint64_t tile, uint32_t len,
                                           uintptr_t ga, uint64_t n, int lane, L& lds,
                                           bool win_only = false, uint32_t mark = ~0u) {
    s.tile = tile;
    s.ga = ga;
    s.len = len;
    s.live = tile * 64 + lane < n;
    // chunks [A & ~15, E) of frames of 64 B .. 64 KiB; longer frames stream
    // their window only (exact checksum path)
    s.shift = (uint32_t)(ga & 15);
    s.wlen = len < ZP_WIN - s.shift ? len : ZP_WIN - s.shift;
    s.giant = len > ZP_GIANT;
    // win_only (the builder's payload frames): the window only, like giants
    const uint32_t span = s.giant || (win_only && len + s.shift > ZP_WIN) ? (uint32_t)ZP_WIN
                                                                          : len + s.shift;
    const uint32_t nch = len >= 64 ? (span + 15) >> 4 : 0u;
    const uint64_t M = __ballot(nch > 0);
    s.ranked = M;
    s.rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32),
                                       __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
    const uint32_t incl = wave_scan(nch);
    const uint32_t pfx = incl - nch;
    const uint32_t T = rdl(incl, 63);
    s.nitems = (T + 63) >> 6;
    // compact the non-empty frames into rank order (ds_permute: LDS untouched)
    const uint32_t nz = (uint32_t)__builtin_popcountll(M);
    const uint32_t dst = nch ? s.rank : nz + ((uint32_t)lane - s.rank);
    const uintptr_t org = (ga & ~(uintptr_t)15) - 16ull * pfx;
    const int a = (int)(dst << 2);
    s.R.org_lo = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)(uint32_t)org);
    s.R.org_hi = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)(uint32_t)(org >> 32));
    s.R.last = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)(incl - 1));
    s.R.pfx = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)pfx);
    // a marked frame offset (T4 streams) inside the streamed chunks
    const uint32_t mc = mark != ~0u && nch ? (s.shift + mark) >> 4 : ~0u;
    const uint32_t mid = mc < nch ? ((pfx + mc) << 4) | ((s.shift + mark) & 15u) : ~0u;
    s.R.mid = (uint32_t)__builtin_amdgcn_ds_permute(a, (int)mid);
    s.cur.rbase = ~0u;
    s.cur.nz = nz;
    s.cur.starts = &lds.starts[0];
    s.run = 0;
}

__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Descriptor loads are unconditional (clamped index, masked after): a load
// count that depends on the lane's branch turns later waits into vmcnt(0).
__device__ __forceinline__ void load_desc(const uint8_t* arena, const uint64_t* offs,
                                          const uint32_t* lens, uint64_t n, uint64_t tile,
                                          int lane, uint32_t& len, uintptr_t& ga) {
    const uint64_t p = tile * 64 + lane;
    const uint64_t pc = p < n ? p : n - 1;
    const uint32_t l = lens[pc];
    const uint64_t o = offs[pc];
    len = p < n ? l : 0u;
    ga = (uintptr_t)arena + (p < n ? o : 0);
}
