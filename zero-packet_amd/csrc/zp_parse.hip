// zp_parse.hip — MI355X (gfx950) batched PacketParser::parse.
//
// Reference path: /root/reference/src/packet/parser.rs:53-140 (parse,
// parse_ipv4, parse_ipv6, parse_protocol) with the readers it calls
// (ethernet.rs:141-212, arp.rs:130-176, ipv4.rs:138-264, ipv6.rs:147-285,
// extensions/headers.rs:51-213, tcp.rs:141-213, udp.rs:103-135,
// icmpv4.rs:92-104, icmpv6.rs:89-101) and the checksum primitives
// (checksum.rs:5-69).
//
// Work decomposition. A tile is 64 consecutive frames on one wave (lane j =
// frame j); waves never synchronise with each other. Per tile:
//   1. descriptors (offs/lens);
//   2. the packed stream: every byte of the tile's frames read once by full
//      1 KiB wave-wide loads (the 16-B chunks of all 64 frames concatenated
//      and cut into items of 64 chunks; see "The stream" below); per-frame
//      sums by running prefix; header windows and last chunks to LDS;
//   3. lane-per-frame header walk from the LDS window;
//   4. checksum verdict, 8-B record store (+ extension chains, if any).
// Checksum arithmetic. The reference verifies S = acc + sum of big-endian
// 16-bit words (u32), valid iff !fold(S) as u16 == 0 (checksum.rs:5-35),
// i.e. S != 0 and S == 0 (mod 65535). We sum little-endian 16-bit words at
// even ARENA addresses (V = E + 256*O, E/O = sums of bytes at even/odd
// addresses) because that is what aligned loads give for free:
//   segment starting at an odd address:  W = V exactly,
//   segment starting at an even address: W == 256*V (mod 65535),
// and W == 0 iff V == 0. Exact u32 sums hold for frames <= 64 KiB; longer
// (IPv6 jumbo) frames take an exact E/O path that reproduces the reference's
// u32 wrap-around. The pseudo-header accumulator is computed exactly from
// E/O sums of the address bytes.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>
#include <mutex>

#include "../../include/zero_packet.h"
#include "../../include/zero_packet_errstr.h"
#include "zp_cols.h"
// Parse-kernel geometry: a 112-B header window (7 KiB of LDS per wave) and
// at most 96 VGPRs, so 18 waves fit a CU instead of 16. Measured per
// placement in one process against the 128-B window at 108 VGPRs: c5 -6 %,
// c3 and c4 within +-1 %.
#define ZP_WIN 112
#define ZP_WPE 5
#include "zp_stream.h"

#define ZP_WAVES 1           // waves per workgroup (independent waves; 1 = finest LDS granularity)
#define ZP_EXT_DENSE 32      // chains per wave from which all 64 ext entries are written
#define ZP_K 1               // consecutive tiles per wave
#define ZP_SMALL_G 4         // tiles of at most this many stream items take one small group (0: off)
#define ZP_TAIL_G 4          // a tile's last <= this many items as one small group (0: off)
// Rejected variants, timing ablations and diagnostic stamps live in
// tools/patches/lab.patch, applied to a scratch copy by
// tools/build_variants.sh (tools/kbench.py --variants); this file is the
// product kernel only.

#ifndef ZP_PARSE_SLOTS_TU
static __thread char g_last_error[256];

static void set_err(const char* what, hipError_t e) {
    snprintf(g_last_error, sizeof g_last_error, "%s: %s", what, hipGetErrorString(e));
}

extern "C" const char* zp_last_error(void) { return g_last_error; }
extern "C" __attribute__((visibility("hidden"))) char* zp__errbuf(void) { return g_last_error; }
extern "C" int zp_abi_version(void) { return ZP_ABI_VERSION; }
extern "C" const char* zp_err_str(int code) { return zp_err_string(code); }
#endif

// --------------------------------------------------------------------------
// Device helpers
// --------------------------------------------------------------------------

// Valid ICMPv4 types (misc.rs:93-119) / ICMPv6 types (misc.rs:164-204).
__device__ __forceinline__ bool icmpv4_type_ok(uint32_t t) {
    const uint64_t m0 = (1ull << 0) | (1ull << 3) | (1ull << 4) | (1ull << 5) | (1ull << 8) |
                        (1ull << 9) | (1ull << 10) | (1ull << 11) | (1ull << 12) | (1ull << 13) |
                        (1ull << 14) | (1ull << 15) | (1ull << 16) | (1ull << 17) | (1ull << 18) |
                        (1ull << 30) | (1ull << 40) | (1ull << 42) | (1ull << 43);
    if (t < 64) return (m0 >> t) & 1;
    return t == 253 || t == 254;
}
__device__ __forceinline__ bool icmpv6_type_ok(uint32_t t) {
    if (t >= 1 && t <= 4) return true;
    if (t == 100 || t == 101 || t == 155 || t == 200 || t == 201) return true;
    return t >= 128 && t <= 153;
}

// --------------------------------------------------------------------------
// Frame view: LDS window (16-B cells, chunk c of frame f at win[c][f ^ c]:
// conflict-free for the cooperative ds_write_b128 of phase A and for each
// lane's ds_read_b128 of its own frame) + global fallback past the window.
// --------------------------------------------------------------------------
// After the stream each lane copies its frame's window cells out
// of the swizzled [chunk][rank] layout into a private contiguous LDS region of
// ZP_RSTRIDE dwords (an odd count: the lanes' reads of one offset fall in 64
// different banks), so a field read is one ds_read_b32 at region + (y >> 2)
// instead of a swizzled-cell address (5 VALU) with 4-way bank conflicts.
#define ZP_RSTRIDE (ZP_WIN / 4 + 1)
struct FrameView {
    const uint4* win;        // this wave's window, [ZP_WIN_CH][64]
    const uint32_t* reg;     // this lane's window, ZP_WIN / 4 dwords from A & ~15
    bool region;             // reg is set (a constant per kernel: the one-frame server reads the cells)
    const uint8_t* g;        // frame in global memory
    uint32_t lane;
    uint32_t shift;          // frame address & 15 (window starts 16-aligned)
    uint32_t wlen;           // frame bytes available in the window
    uint32_t len;            // frame length
    uint4 xc;                // past the window: one cached 16-B chunk ...
    uint32_t xi;             // ... and its index from A & ~15 (~0: none)
    uintptr_t sysbase;       // != 0: the frame lies in the host block at sysbase (system-scope loads)
};

__device__ __forceinline__ uint4 win_chunk(const FrameView& f, uint32_t c) {
    if (f.region) return make_uint4(f.reg[4 * c], f.reg[4 * c + 1], f.reg[4 * c + 2], f.reg[4 * c + 3]);
    return f.win[c * 64 + (f.lane ^ c)];
}
__device__ __forceinline__ uint32_t win_dw(const FrameView& f, uint32_t d) {
    if (f.region) return f.reg[d];
    const uint32_t c = d >> 2;
    return ((const uint32_t*)&f.win[c * 64 + (f.lane ^ c)])[d & 3];
}

// Chunk c (from A & ~15) past the window: one 16-B load per distinct chunk
// (deep IPv6 extension chains and IP-in-IP read a few bytes each from the
// same chunks).
__device__ __forceinline__ uint4 fb_chunk(FrameView& f, uint32_t c) {
    if (c != f.xi) {
        const uintptr_t a = ((uintptr_t)f.g & ~(uintptr_t)15) + 16u * c;
        f.xc = f.sysbase ? ld_sys16(f.sysbase, a) : ldg16(a);
        f.xi = c;
    }
    return f.xc;
}

__device__ __forceinline__ uint32_t dw_of(uint4 v, uint32_t d) {
    return d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
}

__device__ __forceinline__ uint32_t rd8(FrameView& f, uint32_t x) {
    const uint32_t y = x + f.shift;
    const uint32_t dw = x < f.wlen ? win_dw(f, y >> 2) : dw_of(fb_chunk(f, y >> 4), (y >> 2) & 3);
    return (dw >> ((y & 3) * 8)) & 0xFFu;
}

// Big-endian 16-bit field at frame offset x.
__device__ __forceinline__ uint32_t rd16(FrameView& f, uint32_t x) {
    if (x + 1 < f.wlen) {
        const uint32_t y = x + f.shift, d = y >> 2;
        const uint32_t lo = win_dw(f, d);
        const uint32_t hi = (y & 3) == 3 ? win_dw(f, d + 1) : 0u;
        const uint32_t t = __builtin_amdgcn_alignbyte(hi, lo, y & 3);
        return ((t & 0xFFu) << 8) | ((t >> 8) & 0xFFu);
    }
    return (rd8(f, x) << 8) | rd8(f, x + 1);
}

// Masked sums of a 16-B chunk's bytes [l, h): V (LE words at even addresses)
// and B (plain byte sum).
__device__ __forceinline__ void chunk_vb(uint4 v, int l, int h, uint32_t& V, uint32_t& B) {
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t x = (l == 0 && h == 16) ? d[i] : d[i] & byte_mask(4 * i, l, h);
        V = sad16(x, V);
        B = __builtin_amdgcn_sad_u8(x, 0u, B);
    }
}

// V and B over frame bytes [lo, hi) (both <= len): window chunks from LDS,
// chunks past the window through the fallback cache.
template <bool WANT_B>
__device__ __forceinline__ void sum_vb(FrameView& f, uint32_t lo, uint32_t hi, uint32_t& V, uint32_t& B) {
    V = 0;
    B = 0;
    const uint32_t h1 = hi < f.wlen ? hi : f.wlen;
    if (lo < h1) {
        const int ylo = (int)(lo + f.shift), yhi = (int)(h1 + f.shift);
        const int c0 = ylo >> 4, c1 = (yhi - 1) >> 4;
        for (int c = c0; c <= c1; ++c) {
            const int l = c == c0 ? ylo - 16 * c : 0;
            const int h = c == c1 ? yhi - 16 * c : 16;
            if (WANT_B) chunk_vb(win_chunk(f, c), l, h, V, B);
            else V = chunk_sum(win_chunk(f, c), l, h, V);
        }
    }
    const uint32_t l2 = lo > f.wlen ? lo : f.wlen;
    if (l2 < hi) {
        const int ylo = (int)(l2 + f.shift), yhi = (int)(hi + f.shift);
        const int c0 = ylo >> 4, c1 = (yhi - 1) >> 4;
        for (int c = c0; c <= c1; ++c) {
            const int l = c == c0 ? ylo - 16 * c : 0;
            const int h = c == c1 ? yhi - 16 * c : 16;
            if (WANT_B) chunk_vb(fb_chunk(f, (uint32_t)c), l, h, V, B);
            else V = chunk_sum(fb_chunk(f, (uint32_t)c), l, h, V);
        }
    }
}

// Chunk c (from A & ~15) of the frame: the LDS window, then global.
__device__ __forceinline__ uint4 chunk_at(FrameView& f, uint32_t c) {
    return c < ZP_WIN_CH ? win_chunk(f, c) : fb_chunk(f, c);
}

// V-sum of bytes [0, k) of a 16-B chunk (0 <= k <= 16): running v_sad_u16
// over the whole dwords, one bitfield extract for the partial one.
__device__ __forceinline__ uint32_t chunk_prefix(uint4 v, uint32_t k) {
    const uint32_t s1 = sad16(v.x, 0u), s2 = sad16(v.y, s1), s3 = sad16(v.z, s2);
    const uint32_t d = k >> 2;
    const uint32_t full = d == 0 ? 0u : d == 1 ? s1 : d == 2 ? s2 : d == 3 ? s3 : sad16(v.w, s3);
    const uint32_t x = d == 0 ? v.x : d == 1 ? v.y : d == 2 ? v.z : v.w;
    return sad16(__builtin_amdgcn_ubfe(x, 0u, (k & 3u) * 8u), full);
}

// Arena-parity word sum V of frame bytes [lo, hi) (hi <= len): whole chunks
// [c0, c1) plus the prefix of chunk c1 minus the prefix of chunk c0 (no
// per-byte masks; every chunk read holds a byte of the range).
__device__ __forceinline__ uint32_t sumV(FrameView& f, uint32_t lo, uint32_t hi) {
    if (lo >= hi) return 0u;
    const uint32_t ylo = lo + f.shift, yhi = hi + f.shift;
    const uint32_t c0 = ylo >> 4, c1 = (yhi - 1) >> 4;
    uint32_t V = chunk_prefix(chunk_at(f, c1), yhi - 16u * c1) -
                 chunk_prefix(chunk_at(f, c0), ylo & 15u);
    for (uint32_t c = c0; c < c1; ++c) V = chunk_sum(chunk_at(f, c), 0, 16, V);
    return V;
}

// V-sum of the bytes [A & ~15, A + x) (the frame's first x bytes and the
// bytes before it in its first chunk).
__device__ __forceinline__ uint32_t sum_to(FrameView& f, uint32_t x) {
    const uint32_t y = x + f.shift, cx = y >> 4;
    uint32_t V = (y & 15u) ? chunk_prefix(chunk_at(f, cx), y & 15u) : 0u;
    for (uint32_t c = 0; c < cx; ++c) V = chunk_sum(chunk_at(f, c), 0, 16, V);
    return V;
}

// Exact big-endian word sum (reference parity: words start at lo) of frame
// bytes [lo, hi), hi - lo even: with E/O the byte sums at even/odd ARENA
// addresses, V = E + 256*O and B = E + O, so O = (V - B) / 255 exactly; the
// words start at an even address iff A + lo is even.
__device__ __forceinline__ uint32_t sumW_exact(FrameView& f, uint32_t lo, uint32_t hi) {
    uint32_t V, B;
    sum_vb<true>(f, lo, hi, V, B);
    const uint32_t O = (V - B) / 255u, E = B - O;
    return (((uintptr_t)f.g + lo) & 1) ? 256u * O + E : 256u * E + O;
}

// Pseudo-header word sum modulo 65535. For frames of <= 64 KiB the verdict
// (csum_ok) sees the accumulator only as acc mod 65535, and acc >= proto +
// length > 0 (no zero test involved); only jumbo frames, which reproduce the
// reference's u32 wrap-around, need sumW_exact.
__device__ __forceinline__ uint32_t sumW_mod(FrameView& f, uint32_t lo, uint32_t hi) {
    const uint32_t V = sumV(f, lo, hi);
    return (((uintptr_t)f.g + lo) & 1) ? V : V * 256u;   // == W (mod 65535)
}

// Exact reference checksum for long segments: sums even/odd-address bytes
// separately and reproduces the u32 wrap of checksum.rs:12 (release build).
__device__ bool csum_ok_exact(const uint8_t* g, uint32_t lo, uint32_t hi, uint32_t acc) {
    uint64_t E = 0, O = 0;
    const uintptr_t a0 = (uintptr_t)g + lo, a1 = (uintptr_t)g + hi;
    for (uintptr_t d = a0 & ~(uintptr_t)3; d < a1; d += 4) {
        const int l = a0 > d ? (int)(a0 - d) : 0;
        const int h = a1 - d < 4 ? (int)(a1 - d) : 4;
        uint32_t v = ldg4(d) & byte_mask(0, l, h);
        E += (v & 0xFFu) + ((v >> 16) & 0xFFu);
        O += ((v >> 8) & 0xFFu) + (v >> 24);
    }
    uint64_t W = (a0 & 1) ? (256ull * O + E) : (256ull * E + O);
    uint32_t S = (uint32_t)(acc + W);
    while (S >> 16) S = (S & 0xFFFFu) + (S >> 16);
    return (uint16_t)~S == 0;
}

// V of window bytes [a, a + 4M) (window coordinates, a + 4M <= ZP_WIN):
// M + 1 dword reads, two masks, no loop.
template <int M>
__device__ __forceinline__ uint32_t wsum4(const FrameView& f, uint32_t a) {
    const uint32_t d0 = a >> 2, sh = 8u * (a & 3u);
    uint32_t V = sad16(win_dw(f, d0) & (~0u << sh), 0u);
#pragma unroll
    for (int k = 1; k < M; ++k) V = sad16(win_dw(f, d0 + k), V);
    return sad16(win_dw(f, d0 + M) & ~(~0u << sh), V);
}
// Same for a runtime count 1 <= m <= 8 of dwords: one instruction stream
// for the IPv4 (m = 2) and IPv6 (m = 8) pseudo-header addresses of a wave.
// Reads stay inside [d0, d0 + m] (the dwords past m re-read dword m).
__device__ __forceinline__ uint32_t wsum4n(const FrameView& f, uint32_t a, uint32_t m) {
    const uint32_t d0 = a >> 2, sh = 8u * (a & 3u);
    uint32_t V = sad16(win_dw(f, d0) & (~0u << sh), 0u);
#pragma unroll
    for (uint32_t k = 1; k < 8; ++k) {
        const uint32_t x = win_dw(f, d0 + (k < m ? k : m));
        V = sad16(k < m ? x : 0u, V);
    }
    return sad16(win_dw(f, d0 + m) & ~(~0u << sh), V);
}

// --------------------------------------------------------------------------
// The header-chain walk of PacketParser::parse for one frame.
// --------------------------------------------------------------------------
struct Walk {
    zp_rec_full rec;
    uint4 outer;             // ipv6 extension chain as a zp_ext_offsets (valid iff ZP_F_EXT)
    uint4 inner;             // ip_in_ip IPv6 chain (valid iff ZP_F_INNER_EXT)
    uint32_t acc;        // exact pseudo-header accumulator of the innermost IP
    uint32_t l4;         // L4 start (frame offset) when a checksum is pending
    uint8_t pending;     // 1 = L4 checksum still to verify
    uint8_t v6;          // innermost IP is IPv6 (selects the error code)
};

// Slot k's offset into the dwords of a zp_ext_offsets (len in the low half
// of dword 0, off[k] at half k + 1): the chain stays in 4 registers.
__device__ __forceinline__ void put_off(uint32_t (&ed)[4], int slot, uint32_t v) {
#pragma unroll
    for (int k = 0; k < 6; ++k)
        if (k == slot) {
            const int d = (k + 1) >> 1;
            ed[d] = (k & 1) ? (ed[d] & 0xFFFF0000u) | v : (ed[d] & 0xFFFFu) | (v << 16);
        }
}

// Extension-header walk (headers.rs:51-213). Returns 0 or a zp_err.
// pos = IPv6 payload start; outputs slot offsets relative to pos (put_off).
// *code: the chain's inline code (ZP_CHAIN_INLINE, include/zero_packet.h)
// when its headers come in RFC order with lengths the code holds, else 0.
__device__ __forceinline__ int ext_walk(FrameView& f, uint32_t pos, uint32_t nh,
                        uint32_t* present, uint32_t (&ed)[4], uint32_t* total,
                        uint32_t* final_nh, uint32_t* code) {
    uint32_t pres = 0, tot = 0, fin = 0;
    uint32_t cur = nh, p = pos;
    uint32_t cd = ZP_CHAIN_INLINE >> 18, rk = 0;       // rk: RFC rank of the last header + 1
    // One instruction stream for the five header types (Hop-by-Hop :90-113,
    // Routing :117-134, Fragment :138-155, Authentication :159-176,
    // Destination :180-202): a wave whose frames sit on different types runs
    // one step per header, not every type's branch with its own dependent
    // byte read; the next-header and length bytes come in one 16-bit read.
    // Timing-neutral on c3-c6 against per-type branches
    // (profiles/r03_kbench_ext_flat.log), kept as the shorter code.
    for (int it = 0; it < 7; ++it) {                      // <= 6 slots, then a stop
        const bool hbh = cur == 0, rt = cur == 43, fr = cur == 44, ah = cur == 51, ds = cur == 60;
        const uint32_t bit = hbh ? 1u : rt ? 2u : fr ? 4u : ah ? 8u : ds ? ((pres & 16u) ? 32u : 16u) : 0u;
        if (bit == 0 || (pres & bit)) break;              // other header / repeat: Ok (:94-202)
        const uint32_t rem = f.len - p;
        const uint32_t minl = ah ? 12u : 8u;
        const bool opt = hbh || ds;
        if (hbh && pres) return ZP_ERR_EXT_HBH_NOT_FIRST;                 // :98-102
        if (rem < minl)
            return opt ? ZP_ERR_EXT_OPTIONS_TOO_SHORT : rt ? ZP_ERR_EXT_ROUTING_TOO_SHORT
                 : fr ? ZP_ERR_EXT_FRAGMENT_TOO_SHORT : ZP_ERR_EXT_AUTH_TOO_SHORT;
        const uint32_t t = rd16(f, p);                    // next header, header length field
        const uint32_t b1 = t & 0xFFu;
        const uint32_t hl = fr ? 8u : ah ? (b1 + 2) * 4 : (b1 + 1) * 8;
        if (hl > rem)
            return opt ? ZP_ERR_EXT_OPTIONS_EXCEEDS : rt ? ZP_ERR_EXT_ROUTING_EXCEEDS
                       : ZP_ERR_EXT_AUTH_EXCEEDS;
        const int slot = hbh ? ZP_EXT_HBH : rt ? ZP_EXT_RT : fr ? ZP_EXT_FRAG : ah ? ZP_EXT_AH
                       : (bit == 32u ? ZP_EXT_DST2 : ZP_EXT_DST1);
        // inline code: RFC 8200 order HBH, Dest 1st, Routing, Fragment, AH,
        // Dest 2nd (rank 1..6), each length within its code field
        const uint32_t rank = hbh ? 1u : rt ? 3u : fr ? 4u : ah ? 5u : bit == 32u ? 6u : 2u;
        const uint32_t cmax = (hbh || rt) ? 7u : fr ? 0u : 3u;
        const uint32_t sh = hbh ? 0u : rt ? 5u : ah ? 8u : bit == 32u ? 10u : 3u;
        cd = (rank > rk && (fr || b1 <= cmax)) ? cd | (fr ? 0u : b1 << sh) : 0u;
        rk = rank;
        pres |= bit;
        put_off(ed, slot, p - pos);
        tot += hl;
        fin = t >> 8;
        cur = fin;
        p += hl;
    }
    *present = pres;
    *total = tot;
    *final_nh = fin;
    *code = cd;
    return 0;
}

__device__ __forceinline__ void walk_frame(FrameView& f, Walk& w) {
    zp_rec_full& r = w.rec;
    w.pending = 0; w.acc = 0; w.l4 = 0; w.v6 = 0;
    const uint32_t len = f.len;
    int err = 0;
    if (len < 64) { err = ZP_ERR_ETH_FRAME_TOO_SHORT; goto done; }   // parser.rs:159
    {
        uint32_t hl = 14;                                             // ethernet.rs:155-179
        const uint32_t t0 = rd16(f, 12);
        if (t0 == 0x8100) hl = 18;
        else if (t0 == 0x88A8) {
            if (rd16(f, 16) != 0x8100) { err = ZP_ERR_ETH_INVALID_QINQ; goto done; }
            hl = 22;
        }
        r.eth_len = (uint8_t)hl;
        const uint32_t et = rd16(f, hl - 2);                           // ethernet.rs:209-212
        if (et == 0x0806) {                                           // ARP, parser.rs:60,172-180
            if (len - hl < 28) { err = ZP_ERR_ARP_TOO_SHORT; goto done; }
            if (rd16(f, hl + 6) > 2) { err = ZP_ERR_ARP_INVALID_OPER; goto done; }
            r.flags |= ZP_F_ARP;
        } else if (et == 0x0800 || et == 0x86DD) {
            // The IP levels (parse_ipv4 / parse_ipv6 and their IP-in-IP
            // recursion, parser.rs:73-107,134-135) first; the L4 reader and
            // the checksum of the innermost level after the loop, so a wave
            // whose frames end at different levels runs that code once
            // (c5 -5 %).
            uint32_t pos = hl;
            bool v4 = et == 0x0800;
            uint32_t proto, pp;
            for (uint32_t level = 0;; ++level) {
                const uint32_t sl = len - pos;                        // slice length
                if (v4) {                                             // parser.rs:188-212
                    if (sl < 20) { err = ZP_ERR_IPV4_TOO_SHORT; goto done; }
                    const uint32_t b0 = rd8(f, pos);
                    if ((b0 >> 4) != 4) { err = ZP_ERR_IPV4_VERSION; goto done; }
                    const uint32_t ihl = (b0 & 15) * 4;
                    if (ihl < 20) { err = ZP_ERR_IPV4_IHL_TOO_SHORT; goto done; }
                    if (sl < ihl) { err = ZP_ERR_IPV4_HDR_TOO_LONG; goto done; }
                    if (rd16(f, pos + 2) != sl) { err = ZP_ERR_IPV4_TOTAL_LENGTH; goto done; }
                    // ipv4.rs:262-264; a 20-B header inside the window (the
                    // common case) straight-line (c5 -4 %)
                    const uint32_t hv = (ihl == 20 && pos + 20 <= f.wlen)
                                            ? wsum4<5>(f, pos + f.shift) : sumV(f, pos, pos + ihl);
                    if (!nz_mod65535_zero(hv)) { err = ZP_ERR_IPV4_CHECKSUM; goto done; }
                    proto = rd8(f, pos + 9);
                    pp = pos + ihl;
                    if (level == 0) r.flags |= ZP_F_IPV4;
                    else if (level == 1) { r.flags |= ZP_F_IP_IN_IP; r.inner_off = pos; }
                } else {                                              // parser.rs:222-230
                    if (sl < 40) { err = ZP_ERR_IPV6_TOO_SHORT; goto done; }
                    uint32_t pres = 0, tot = 0, fin = 0, cd = 0;
                    uint32_t eo[4] = {0, 0, 0, 0};
                    const uint32_t nh = rd8(f, pos + 6);
                    const int e = ext_walk(f, pos + 40, nh, &pres, eo, &tot, &fin, &cd);  // ipv6.rs:159
                    if (e) { err = e; goto done; }
                    if ((rd8(f, pos) >> 4) != 6) { err = ZP_ERR_IPV6_VERSION; goto done; }
                    proto = pres ? fin : nh;                          // ipv6.rs:219-227
                    pp = pos + 40 + tot;                              // ipv6.rs:283-285
                    if (level == 0) {
                        r.flags |= ZP_F_IPV6;
                        r.final_nh = (uint8_t)proto;
                        if (pres) {
                            r.flags |= ZP_F_EXT | (pres << 12);
                            r.chain = cd;
                            // final_next_header (headers.rs:26) in byte 14
                            w.outer = make_uint4(eo[0] | tot, eo[1], eo[2], eo[3] | (proto << 16));
                        }
                    } else if (level == 1) {
                        r.flags |= ZP_F_IP_IN_IP | ZP_F_IP_IN_IP_V6;
                        r.inner_off = pos;
                        r.inner_final_nh = (uint8_t)proto;
                        if (pres) {
                            r.flags |= ZP_F_INNER_EXT | (pres << 18);
                            w.inner = make_uint4(eo[0] | tot, eo[1], eo[2], eo[3] | (proto << 16));
                        }
                    }
                }
                if (proto != 4 && proto != 41) break;                 // parse_protocol :111-140
                v4 = proto == 4;                                      // IP-in-IP recursion
                pos = pp;
            }
            {
                const uint32_t rem = len - pp;                        // parse_protocol :111-140
                const bool tcp = proto == 6, udp = proto == 17, ic4 = proto == 1;
                if (tcp || udp || ic4 || proto == 58) {
                    // One code path for the four L4 readers (no divergent
                    // duplicate per type): each reads one 16-bit word, at
                    // +12 (TCP data offset/flags), +4 (UDP length) or +0
                    // (ICMP type/code); the checks and error codes per type
                    // are those of tcp.rs:141-147 / parser.rs:237-247,
                    // udp.rs:103-107 / parser.rs:258-263, icmpv4.rs:92-97 /
                    // parser.rs:273-283, icmpv6.rs:89-94 / parser.rs:293-299.
                    if (rem < (tcp ? 20u : 8u)) {
                        err = tcp ? ZP_ERR_TCP_TOO_SHORT
                                  : udp ? ZP_ERR_UDP_TOO_SHORT : ZP_ERR_ICMP_TOO_SHORT;
                        goto done;
                    }
                    const uint32_t t = rd16(f, pp + (tcp ? 12u : udp ? 4u : 0u));
                    int e;
                    if (tcp) e = (t >> 12) * 4 < 20 ? ZP_ERR_TCP_DATA_OFFSET
                               : (t & 0xFF) == 0 ? ZP_ERR_TCP_FLAGS : 0;
                    else if (udp) e = t != rem ? ZP_ERR_UDP_LENGTH : 0;
                    else if (ic4) e = !icmpv4_type_ok(t >> 8) ? ZP_ERR_ICMPV4_TYPE
                                    : (t & 0xFF) > 15 ? ZP_ERR_ICMPV4_CODE : 0;
                    else e = !icmpv6_type_ok(t >> 8) ? ZP_ERR_ICMPV6_TYPE : 0;
                    if (e) { err = e; goto done; }
                    r.flags |= tcp ? ZP_F_TCP : udp ? ZP_F_UDP : ic4 ? ZP_F_ICMPV4 : ZP_F_ICMPV6;
                } else {
                    goto ip_done;                                     // unknown: Ok, no L4
                }
                // Pseudo-header of the innermost IP only (outer levels of an
                // IP-in-IP chain never need one): parser.rs:316-333 (IPv4;
                // none for ICMPv4), parser.rs:341-361 (IPv6, final next header).
                // One pseudo-header sum for both IP versions (the address range differs,
                // the code does not: no divergent duplicate).
                const uint32_t plo = v4 ? pos + 12 : pos + 8, phi = v4 ? pos + 20 : pos + 40;
                uint32_t ps;
                if (len > ZP_GIANT) ps = sumW_exact(f, plo, phi);
                else if (phi <= f.wlen) {                             // in the window:
                    const uint32_t V = wsum4n(f, plo + f.shift, v4 ? 2u : 8u);  // straight-line
                    ps = (((uintptr_t)f.g + plo) & 1) ? V : V * 256u;   // (c5 -1 %)
                }
                else ps = sumW_mod(f, plo, phi);
                w.acc = (v4 && proto == 1) ? 0u : ps + proto + (len - pp);
                r.l4_off = pp;
                w.pending = 1;
                w.l4 = pp;
                w.v6 = v4 ? 0 : 1;
            }
        }
    ip_done:
        r.flags |= ZP_F_ETHERNET;
    }
done:
    if (err) {
        r = zp_rec_full{};
        r.err = (uint8_t)err;
        w.pending = 0;
    }
}

// Byte reader over a FrameView for the fused column views (zp_cols.h): the
// LDS window, then the walk's one-chunk cache past it (c4 fused −4 % against
// plain global byte loads; no stack frame since the walk helpers are
// force-inlined).
struct ViewReader {
    FrameView& f;
    __device__ __forceinline__ uint32_t operator()(uint32_t x) { return rd8(f, x); }
    __device__ __forceinline__ bool has4(uint32_t x) const { return x + 3 < f.wlen; }
    __device__ __forceinline__ uint32_t le4(uint32_t x) const {
        const uint32_t y = x + f.shift, d = y >> 2;
        const uint32_t lo = win_dw(f, d), hi = (y & 3) ? win_dw(f, d + 1) : 0u;
        return __builtin_amdgcn_alignbyte(hi, lo, y & 3);
    }
};

// --------------------------------------------------------------------------
// The common frame, straight-line: Ethernet II without tags, IPv4 with a
// 20-B header, TCP / UDP / ICMPv4 (c1-c3, most real traffic). Every field of
// that shape lies in the first 48 bytes, inside the LDS window, so the reads
// need no bound checks and the sums no loops. fast_v4 accepts a frame only
// when the general walk would accept it with exactly these readers (every
// check of parser.rs:153-287 on this path passes); anything else (other
// shapes, any failing check) takes the general walk, which then finds the
// first error in the reference's order.
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wb8(const FrameView& f, uint32_t x) {
    const uint32_t y = x + f.shift;
    return (win_dw(f, y >> 2) >> ((y & 3) * 8)) & 0xFFu;
}
__device__ __forceinline__ uint32_t wbe16(const FrameView& f, uint32_t x) {
    const uint32_t y = x + f.shift, d = y >> 2;
    const uint32_t t = __builtin_amdgcn_alignbyte(win_dw(f, d + 1), win_dw(f, d), y & 3);
    return ((t & 0xFFu) << 8) | ((t >> 8) & 0xFFu);
}
// The first header fields every straight-line path tests, read from the
// window once per frame (ethernet.rs:155-179: the tag types, the header
// length, the ethertype; the IP version / IHL byte and the IPv6 next header).
struct Probe { uint32_t t0, t1, hl, et, b0, p6; };
__device__ __forceinline__ Probe probe_frame(const FrameView& f) {
    Probe p;
    p.t0 = wbe16(f, 12);
    p.t1 = wbe16(f, 16);
    p.hl = p.t0 == 0x8100 ? 18u : p.t0 == 0x88A8 ? 22u : 14u;
    p.et = wbe16(f, p.hl - 2);
    p.b0 = wb8(f, p.hl);
    p.p6 = wb8(f, p.hl + 6);
    return p;
}
// The frame looks like the common shape (untagged Ethernet II, IPv4 IHL 5).
__device__ __forceinline__ bool v4_probe(const FrameView& f, const Probe& p) {
    return f.len >= 64 && p.t0 == 0x0800 && p.b0 == 0x45;
}
__device__ __forceinline__ bool fast_v4(const FrameView& f, const Probe& pr, Walk& w) {
    const uint32_t len = f.len;
    const uint32_t hv = wsum4<5>(f, 14 + f.shift);                  // ipv4.rs:262-264
    const uint32_t proto = wb8(f, 23);
    const bool tcp = proto == 6, udp = proto == 17, ic4 = proto == 1;
    const uint32_t t = wbe16(f, tcp ? 46u : udp ? 38u : 34u);       // one L4 word
    bool ok = v4_probe(f, pr) && pr.t1 == len - 14 &&              // parser.rs:188-212
              nz_mod65535_zero(hv) && (tcp || udp || ic4);
    ok = ok && (tcp ? (t >> 12) >= 5 && (t & 0xFFu) != 0             // parser.rs:237-247
              : udp ? t == len - 34                                  // parser.rs:258-263
                    : icmpv4_type_ok(t >> 8) && (t & 0xFFu) <= 15);  // parser.rs:273-283
    const uint32_t pv = wsum4<2>(f, 26 + f.shift);                  // addresses, checksum.rs:38-63
    const uint32_t ps = (((uintptr_t)f.g + 26) & 1) ? pv : pv * 256u;
    w.acc = ic4 ? 0u : ps + proto + (len - 34);                     // parser.rs:316-333
    w.rec.flags = ZP_F_ETHERNET | ZP_F_IPV4 | (tcp ? ZP_F_TCP : udp ? ZP_F_UDP : ZP_F_ICMPV4);
    w.rec.eth_len = 14;
    w.rec.l4_off = 34;
    w.l4 = 34;
    w.pending = 1;
    w.v6 = 0;
    return ok;
}

// --------------------------------------------------------------------------
// The common stacks of mixed traffic, straight-line (c5, c6): Ethernet with
// 0, 1 (802.1Q) or 2 (Q-in-Q) tags; IPv4 with a 20-B header or IPv6 without
// extension headers; at most one IP-in-IP level, either version in either;
// TCP / UDP / ICMPv4 / ICMPv6 or a protocol without an L4 reader. Both IP
// versions of a level are read and checked in one instruction stream and
// selected (no divergent v4 / v6 branches, no level loop), so a wave of
// mixed stacks runs one short path instead of every branch of walk_frame.
// Like fast_v4 it accepts a frame only when walk_frame would accept it with
// exactly these readers and this record; any other frame (other stacks, any
// failing check) is left to walk_frame, which finds the reference's first
// error. Every header field it reads lies in the window, except the L4 word
// and the pseudo-header addresses of a deep stack, which take the
// window-or-global readers. The highest byte read from the window is 81: the
// encapsulated IPv4 header sum (wsum4<5>, bytes [62, 82)) behind Q-in-Q (22)
// + IPv6 (40). The window holds min(len, ZP_WIN - 15) bytes of a frame, so
// every frame of >= 82 bytes has them there; a shorter one fails that
// level's `pos + 20 <= len` check whatever the bytes past it hold.
// --------------------------------------------------------------------------
static_assert(ZP_WIN - 15 >= 82, "fast_ip reads frame bytes up to 81 from the window");
struct IpLevel { uint32_t proto, next; bool ok; };
// One IP level at `pos` (parser.rs:188-212 with a 20-B header / 222-230
// without extension headers), both versions computed, `v4` selecting.
__device__ __forceinline__ IpLevel ip_level(const FrameView& f, uint32_t pos, bool v4) {
    const uint32_t sl = f.len - pos;
    const uint32_t b0 = wb8(f, pos);
    const uint32_t tl = wbe16(f, pos + 2);
    const uint32_t p4 = wb8(f, pos + 9), p6 = wb8(f, pos + 6);
    const uint32_t hv = wsum4<5>(f, pos + f.shift);                      // ipv4.rs:262-264
    const bool ok4 = pos + 20 <= f.len && b0 == 0x45 && tl == sl && nz_mod65535_zero(hv);
    const bool ext6 = p6 == 0 || p6 == 43 || p6 == 44 || p6 == 51 || p6 == 60;  // headers.rs:73-86
    const bool ok6 = pos + 40 <= f.len && (b0 >> 4) == 6 && !ext6;
    IpLevel L;
    L.ok = v4 ? ok4 : ok6;
    L.proto = v4 ? p4 : p6;
    L.next = pos + (v4 ? 20u : 40u);
    return L;
}
// Frames fast_ip can take, by their first headers: a wave with any frame it
// surely cannot take (ARP, IPv4 options, IPv6 extension headers, runts)
// skips it, since the general walk then runs for the wave anyway (c6 +1.5 %
// without this gate).
__device__ __forceinline__ bool fast_ip_probe(const FrameView& f, const Probe& p) {
    if (f.len < 64) return false;
    const bool ext6 = p.p6 == 0 || p.p6 == 43 || p.p6 == 44 || p.p6 == 51 || p.p6 == 60;
    return p.et == 0x0800 ? p.b0 == 0x45 : p.et == 0x86DD && !ext6;
}
__device__ __forceinline__ bool fast_ip(FrameView& f, const Probe& pr, Walk& w) {
    const uint32_t len = f.len;
    if (len < 64 || len > ZP_GIANT) return false;
    const uint32_t t0 = pr.t0, t1 = pr.t1;                              // ethernet.rs:155-179
    const uint32_t hl = pr.hl;
    const uint32_t et = pr.et;                                          // ethernet.rs:209-212
    const bool v4o = et == 0x0800;
    bool ok = (t0 != 0x88A8 || t1 == 0x8100) && (v4o || et == 0x86DD);
    const IpLevel L0 = ip_level(f, hl, v4o);                            // parse_ipv4 / parse_ipv6
    const bool enc = L0.proto == 4 || L0.proto == 41;                   // parser.rs:134-135
    const bool v4i = L0.proto == 4;
    const IpLevel L1 = ip_level(f, L0.next, v4i);
    ok = ok && L0.ok && (!enc || (L1.ok && L1.proto != 4 && L1.proto != 41));
    const uint32_t proto = enc ? L1.proto : L0.proto;
    const uint32_t pp = enc ? L1.next : L0.next;
    const uint32_t ipl = enc ? L0.next : hl;                            // innermost IP header
    const bool v4 = enc ? v4i : v4o;
    // parse_protocol (parser.rs:111-140): the L4 reader of the protocol
    const uint32_t rem = len - pp;
    const bool tcp = proto == 6, udp = proto == 17, ic4 = proto == 1, ic6 = proto == 58;
    const bool l4 = tcp || udp || ic4 || ic6;
    if (ok && l4) {
        ok = rem >= (tcp ? 20u : 8u);
        if (ok) {
            const uint32_t t = rd16(f, pp + (tcp ? 12u : udp ? 4u : 0u));
            ok = tcp ? (t >> 12) >= 5 && (t & 0xFFu) != 0                 // parser.rs:237-247
               : udp ? t == rem                                            // parser.rs:258-263
               : ic4 ? icmpv4_type_ok(t >> 8) && (t & 0xFFu) <= 15         // parser.rs:273-283
                     : icmpv6_type_ok(t >> 8);                             // parser.rs:293-299
        }
    }
    zp_rec_full& r = w.rec;
    r.flags = ZP_F_ETHERNET | (v4o ? ZP_F_IPV4 : ZP_F_IPV6) |
              (enc ? ZP_F_IP_IN_IP | (v4i ? 0u : ZP_F_IP_IN_IP_V6) : 0u) |
              (tcp ? ZP_F_TCP : udp ? ZP_F_UDP : ic4 ? ZP_F_ICMPV4 : ic6 ? ZP_F_ICMPV6 : 0u);
    r.eth_len = (uint8_t)hl;
    r.final_nh = v4o ? 0 : (uint8_t)L0.proto;                           // ipv6.rs:219-227
    r.inner_final_nh = enc && !v4i ? (uint8_t)L1.proto : 0;
    r.inner_off = enc ? L0.next : 0u;
    r.l4_off = l4 ? pp : 0u;
    w.pending = l4;
    w.l4 = pp;
    w.v6 = v4 ? 0 : 1;
    w.acc = 0;
    if (ok && l4 && !(v4 && ic4)) {
        // pseudo-header of the innermost IP (parser.rs:316-333, 341-361)
        const uint32_t plo = v4 ? ipl + 12 : ipl + 8, phi = v4 ? ipl + 20 : ipl + 40;
        uint32_t ps;
        if (phi <= f.wlen) {
            const uint32_t V = wsum4n(f, plo + f.shift, v4 ? 2u : 8u);
            ps = (((uintptr_t)f.g + plo) & 1) ? V : V * 256u;
        } else {
            ps = sumW_mod(f, plo, phi);
        }
        w.acc = ps + proto + rem;
    }
    return ok;
}

// --------------------------------------------------------------------------
// Minimum-size frames in registers. A tile whose live frames are all 64 B
// (the Ethernet minimum; c1/c2, line-rate small-packet traffic) does not need
// the packed stream, the LDS window or the walk: each lane loads its own
// frame (4 dwordx4 + 1 dword from A & ~3: never past the 16-B chunk holding
// the frame's last byte, as the stream), aligns it to 16 frame dwords, and
// checks the common shape (Ethernet II / IPv4 with a 20-B header / TCP, UDP,
// ICMPv4) with both checksums from the registers. Word sums are taken at even
// FRAME offsets, little-endian: a big-endian word w is 256 * (its LE value)
// mod 65535, and a sum is zero iff all its words are, so the checks of
// csum_ok hold with `odd` = false. If any live lane's frame is not of that
// shape or fails a check, the tile takes the stream path, whose walk finds
// the reference's first error.
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t tiny_be16(const uint32_t (&f)[16], uint32_t x) {
    const uint32_t d = f[x >> 2] >> (8 * (x & 2));                 // x even
    return ((d & 0xFFu) << 8) | ((d >> 8) & 0xFFu);
}
// Record codes (round 6). Inside the read stream a record store costs the
// stream in proportion to the contiguous bytes a wave stores: 64 x 8 B
// +0.23 ms on c3, 64 B per tile +0.044 (DESIGN.md §4,
// profiles/r06_rec_slot_probe.log). A full tile whose 64 records all have
// the common form (no error, no IP-in-IP, no extension headers, Ethernet
// code 0-2, the L4 reader right after a 20-B IPv4 or 40-B IPv6 header)
// stores one byte per frame over its first 8 records instead, and
// zp_rec_expand_kernel rewrites the tile's 64 records from them after the
// parse (write-only, ~0.03 ms on c3). Code = 0xC0 + 15 * eth_code + 5 * l3
// + l4 (l3: ARP / IPv4 / IPv6, l4: none / TCP / UDP / ICMPv4 / ICMPv6):
// byte 3 of a tile's first record is <= 0x97 (err <= 37), of a code tile
// >= 0xC0. Any other tile (a record without a code, a partial last tile,
// the fused column kernel, the zp_parse_one server) stores its records.
#define ZP_CODE_BASE 0xC0u
__device__ __forceinline__ uint32_t rec_code(zp_u32x2 pk) {
    const uint32_t f = pk.x, ec = (f >> 24) & 3u;
    const uint32_t l3 = (f & ZP_F_ARP) ? 0u : (f & ZP_F_IPV4) ? 1u : (f & ZP_F_IPV6) ? 2u : 3u;
    const uint32_t l4 = (f & ZP_F_TCP) ? 1u : (f & ZP_F_UDP) ? 2u : (f & ZP_F_ICMPV4) ? 3u
                      : (f & ZP_F_ICMPV6) ? 4u : 0u;
    const uint32_t want = ZP_F_ETHERNET | (l3 == 0 ? ZP_F_ARP : l3 == 1 ? ZP_F_IPV4 : ZP_F_IPV6) |
                          (l4 == 1 ? ZP_F_TCP : l4 == 2 ? ZP_F_UDP : l4 == 3 ? ZP_F_ICMPV4
                           : l4 == 4 ? ZP_F_ICMPV6 : 0u);
    const uint32_t off = l4 ? 14u + 4u * ec + (l3 == 1 ? 20u : 40u) : 0u;
    const bool ok = ec < 3u && l3 < 3u && (l3 != 0 || l4 == 0) && (f & 0xFCFFFFFFu) == want &&
                    pk.y == off;
    return ok ? ZP_CODE_BASE + 15u * ec + 5u * l3 + l4 : 0u;
}
// The record of a code (zp_rec_expand_kernel).
__device__ __forceinline__ zp_u32x2 code_rec(uint32_t c) {
    const uint32_t x = c - ZP_CODE_BASE, ec = x / 15u, l3 = x / 5u % 3u, l4 = x % 5u;
    const uint32_t f = ZP_F_ETHERNET | (l3 == 0 ? ZP_F_ARP : l3 == 1 ? ZP_F_IPV4 : ZP_F_IPV6) |
                       (l4 == 1 ? ZP_F_TCP : l4 == 2 ? ZP_F_UDP : l4 == 3 ? ZP_F_ICMPV4
                        : l4 == 4 ? ZP_F_ICMPV6 : 0u) | ec << 24;
    return zp_u32x2{f, l4 ? 14u + 4u * ec + (l3 == 1 ? 20u : 40u) : 0u};
}


__device__ __forceinline__ bool tiny_tile(uint64_t tile, uint32_t len, uintptr_t ga, uint64_t n,
                                          int lane, zp_record* __restrict__ records, bool slots) {
    const bool live = tile * 64 + lane < n;
    const uintptr_t base = ga & ~(uintptr_t)3;
    const uint32_t sh = (uint32_t)(ga & 3);
    uint32_t w[17];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const zp_u32x4 q = *(const ZP_GLOBAL zp_u32x4*)(live ? base + 16 * k : ga);
        w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
    }
    w[16] = (live && sh) ? *(const ZP_GLOBAL uint32_t*)(base + 64) : 0u;
    uint32_t f[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) f[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
    // parser.rs:153-165, 188-212 (IPv4, IHL 5), then the L4 reader of the
    // protocol (parser.rs:237-283) and the checksum (parser.rs:316-333)
    const uint32_t proto = f[5] >> 24;
    const bool tcp = proto == 6, udp = proto == 17, ic4 = proto == 1;
    const uint32_t hv = sad16(f[3] >> 16, sad16(f[4], sad16(f[5], sad16(f[6], sad16(f[7],
                            sad16(f[8] & 0xFFFFu, 0u))))));            // bytes 14..33
    const uint32_t t = tiny_be16(f, tcp ? 46u : udp ? 38u : 34u);
    bool ok = tiny_be16(f, 12) == 0x0800 && ((f[3] >> 16) & 0xFFu) == 0x45 &&
              tiny_be16(f, 16) == 50u && nz_mod65535_zero(hv) && (tcp || udp || ic4);
    ok = ok && (tcp ? (t >> 12) >= 5 && (t & 0xFFu) != 0
              : udp ? t == 30u
                    : icmpv4_type_ok(t >> 8) && (t & 0xFFu) <= 15);
    const uint32_t pv = sad16(f[6] >> 16, sad16(f[7], sad16(f[8] & 0xFFFFu, 0u)));  // 26..33
    const uint32_t ps = (pv % 65535u) * 256u;                          // BE address words
    const uint32_t acc = ic4 ? 0u : ps + proto + 30u;
    uint32_t lv = sad16(f[8] >> 16, 0u);                               // L4 bytes 34..63
#pragma unroll
    for (int k = 9; k < 16; ++k) lv = sad16(f[k], lv);
    ok = ok && csum_ok(acc, lv, false);
    if (__ballot(live && !ok)) return false;                           // wave-uniform
    if (slots && tile * 64 + 64 <= n) {                               // every lane live: codes
        const uint32_t c = ZP_CODE_BASE + 5u + (tcp ? 1u : udp ? 2u : 3u);   // code 0, IPv4
        __builtin_nontemporal_store((uint8_t)c, (uint8_t*)(records + tile * 64) + lane);
        return true;
    }
    if (live) {
        // Ethernet II (code 0), IPv4, the L4 reader at 34
        const uint32_t flags = ZP_F_ETHERNET | ZP_F_IPV4 | (tcp ? ZP_F_TCP : udp ? ZP_F_UDP : ZP_F_ICMPV4);
        __builtin_nontemporal_store(zp_u32x2{flags, 34u}, (zp_u32x2*)(records + tile * 64 + lane));
    }
    return true;
}

__device__ __forceinline__ void store_ext(zp_ext_offsets* base, uint64_t i, uint4 q) {
    __builtin_nontemporal_store(zp_u32x4{q.x, q.y, q.z, q.w}, (zp_u32x4*)(base + i));
}

// Header walk + checksum verdict + record store of a streamed tile; with COLS
// also the column views, from the same LDS window (no second pass).
template <bool COLS, bool SYS = false, class L = WaveLds, bool SLOTS = false>
__device__ __forceinline__ void tile_finish(TileState& s, uint64_t n, int lane, L& lds,
                                            zp_record* __restrict__ records,
                                            zp_ext_offsets* __restrict__ ext,
                                            const ColPtrs& cols, uintptr_t sysbase = 0,
                                            zp_u32x2* sys_rec = nullptr) {
    constexpr bool TAILS = sizeof(lds.win) > sizeof(uint4) * ZP_WIN_CH * 64;   // last-chunk cells
    static_assert(TAILS || !SYS, "the tail-free layout needs the region path");
    uint4* tail = TAILS ? &lds.win[0] + ZP_WIN_CH * 64 : nullptr;
    const uint8_t* g = (const uint8_t*)s.ga;
    // the frame's stream sum (before the regions overlay the running sums)
    const uint32_t fsum = lds.cend[s.rank & 63u] - ((s.rank & 63u) ? lds.cend[(s.rank & 63u) - 1u] : 0u);
    FrameView fv;
    fv.win = &lds.win[0];
    fv.g = g;
    fv.lane = s.rank & 63u;
    fv.shift = s.shift;
    fv.len = s.len;
    fv.wlen = s.wlen;
    fv.xc = make_uint4(0, 0, 0, 0);
    fv.xi = ~0u;
    fv.sysbase = SYS ? sysbase : 0;
    // the frame's cells and last chunk to registers, then its window to the
    // lane's private region (it overlays the cells and part of the tails);
    // the one-frame tile of the zp_parse_one server (SYS) reads the cells
    // where the stream put them (the copy is latency on its critical path)
    uint4 mytail;
    fv.region = !SYS;
    if (SYS) {
        mytail = tail[s.rank & 63u];
        fv.reg = nullptr;
    } else {
        static_assert(64 * ZP_RSTRIDE * 4 <= sizeof(L), "regions fit the wave's LDS");
        const uint32_t rk = s.rank & 63u;
        uint4 cell[ZP_WIN_CH];
#pragma unroll
        for (uint32_t c = 0; c < ZP_WIN_CH; ++c) cell[c] = lds.win[c * 64 + ((rk ^ c) & 63u)];
        mytail = tail[rk];
        wave_lds_fence();
        uint32_t* reg = (uint32_t*)&lds.win[0] + (uint32_t)lane * ZP_RSTRIDE;
#pragma unroll
        for (uint32_t c = 0; c < ZP_WIN_CH; ++c) {
            reg[4 * c] = cell[c].x; reg[4 * c + 1] = cell[c].y;
            reg[4 * c + 2] = cell[c].z; reg[4 * c + 3] = cell[c].w;
        }
        wave_lds_fence();
        fv.reg = reg;
    }
    Walk w;
    w.rec = zp_rec_full{};
    w.outer = make_uint4(0, 0, 0, 0);
    w.inner = make_uint4(0, 0, 0, 0);
    bool done = false;
    const Probe pr = probe_frame(fv);          // the first header fields, read once
    // The common shape straight-line when most of the wave has it
    // (wave-uniform test); the rest of the frames take the general walk.
    const bool probe = s.live && v4_probe(fv, pr);
    // (SYS: the one-frame tile of the zp_parse_one server takes it alone)
    if (__builtin_popcountll(__ballot(probe)) >= (SYS ? 1 : 32)) {
        if (probe) done = fast_v4(fv, pr, w);
    }
    // Mixed stacks straight-line (c5 -5.5 %); what it leaves takes the
    // general walk.
    {
        const bool todo = s.live && !done;
        if (__ballot(todo) && !__ballot(todo && !fast_ip_probe(fv, pr))) {
            if (todo) done = fast_ip(fv, pr, w);
        }
    }
    if (__ballot(s.live && !done)) {
        if (s.live && !done) {
            w.rec = zp_rec_full{};
            walk_frame(fv, w);
        }
    }
    if (!s.live) return;
    // The frame's stream sum covers the whole chunks [A & ~15, E16):
    // L4 sum = that - V[A & ~15, A + l4) - V[E, E16).
    zp_rec_full rec = w.rec;
    const uint64_t p = s.tile * 64 + lane;
    // A full tile whose walk records all have codes stores after the verdict
    // (wave-uniform: all 64 lanes are live only in a full tile).
    // (a flags test first: a tile with an error, a tunnel or a chain skips
    // the code arithmetic)
    const bool slot = SLOTS && !SYS && !COLS && __ballot(true) == ~0ull &&
                      !__ballot((zp_pack(rec).x & (0xFC000000u | ZP_F_IP_IN_IP | ZP_F_EXT | ZP_F_INNER_EXT)) != 0u) &&
                      !__ballot(rec_code(zp_pack(rec)) == 0u);
    // Otherwise the record as the walk left it goes out before the verdict,
    // so its store's latency overlaps the checksum work instead of ending
    // the wave (two boxes: c5 -1.6 / -0.6 %, c3 -0.3 / +0.6 %, c4 -0.4 /
    // +0.3 %; profiles/r05_kbench_early_rec.log,
    // r05_kbench_early_rec_k2_norec.log); a frame whose L4 checksum then
    // fails stores its error record over it (same lane, same address: the
    // later store lands last).
    if (!SYS && !slot) __builtin_nontemporal_store(zp_pack(rec), (zp_u32x2*)(records + p));
    if (w.pending) {
        bool ok;
        if (s.giant) {
            ok = csum_ok_exact(g, w.l4, s.len, w.acc);
        } else {
            const bool odd = (s.ga + w.l4) & 1;
            const uint32_t he = (s.len + s.shift) & 15u;    // bytes of the last chunk in use
            const uint32_t ex = he ? range_sum(mytail, he, 16u) : 0u;
            ok = csum_ok(w.acc, fsum - sum_to(fv, w.l4) - ex, odd);
        }
        if (!ok) {
            rec = zp_rec_full{};
            rec.err = (uint8_t)(w.v6 ? ZP_ERR_IPV6_L4_CHECKSUM : ZP_ERR_IPV4_L4_CHECKSUM);
            if (!SYS && !slot) __builtin_nontemporal_store(zp_pack(rec), (zp_u32x2*)(records + p));
        }
    }
    // Records are nontemporal 8-B stores, one per frame (512 B of whole
    // lines per wave instruction): nt took 6-7 % off on every placement,
    // 16-B records (v2) 4-6 % against 32-B ones, 8-B records (v4) 2-7 % more.
    static_assert(sizeof(zp_record) == 8 && sizeof(zp_ext_offsets) == 16, "8-B records");
    if (slot) {
        // the final records (a failed checksum has no code): codes if every
        // frame still has one, else every lane's record
        const zp_u32x2 pk = zp_pack(rec);
        const uint32_t c = rec_code(pk);
        if (!__ballot(c == 0u))
            __builtin_nontemporal_store((uint8_t)c, (uint8_t*)(records + s.tile * 64) + lane);
        else
            __builtin_nontemporal_store(pk, (zp_u32x2*)(records + p));
    }
    // the server stores it with its acknowledgement (one 16-B store)
    if (SYS) *sys_rec = zp_pack(rec);
    if (ext) {
        // The extension chains: a wave with at least ZP_EXT_DENSE chains
        // writes the entries of all its frames (whole lines, zero where
        // absent), one with fewer only those of its chains. Measured on tiles
        // of k chained frames among IPv4 frames (tools/mix_probe.py): only
        // the flagged entries is faster up to k = 24 (-2.4 %), equal at 32,
        // slower from 48 (c4, 56 per wave: +3 %). Nontemporal like the
        // records (c4 -1.3 %, c6 -2.1 %).
        // an inline outer chain (ABI v6) has no entry
        const bool ho = (rec.flags & ZP_F_EXT) && !zp_chain_inline(rec),
                   hi = rec.flags & ZP_F_INNER_EXT;
        const uint64_t mo = __ballot(ho), mi = __ballot(hi);
        if (SYS) {                                        // one frame: its own entries
            if (ho) st_sys16(sysbase, (uintptr_t)(ext + p),
                             zp_u32x4{w.outer.x, w.outer.y, w.outer.z, w.outer.w});
            if (hi) st_sys16(sysbase, (uintptr_t)(ext + n + p),
                             zp_u32x4{w.inner.x, w.inner.y, w.inner.z, w.inner.w});
            // the entries are in host memory before the record and its
            // acknowledgement go out (a store's completion is one host-link
            // round trip: frames without entries skip it)
            if (ho || hi) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
        if (mo && (ho || __builtin_popcountll(mo) >= ZP_EXT_DENSE))
            store_ext(ext, p, ho ? w.outer : make_uint4(0, 0, 0, 0));
        if (mi && (hi || __builtin_popcountll(mi) >= ZP_EXT_DENSE))
            store_ext(ext, n + p, hi ? w.inner : make_uint4(0, 0, 0, 0));
        }
    }
    if (COLS) {
        ViewReader rdr{fv};
        emit_columns(rdr, rec, rec.err == 0 && (rec.flags & ZP_F_ETHERNET), s.len, p, cols);
    }
}


// One wave per tile; the hardware back-fills finished waves with the next
// tiles in dispatch order, so the resident waves always stream a contiguous
// band of the arena (measured: a persistent grid looping over tiles was
// 9-12 % slower on c3/c5).
#define ZP_KATTR __launch_bounds__(64 * ZP_WAVES) __attribute__((amdgpu_waves_per_eu(ZP_WPE)))
// The fused parse + columns kernel carries the column getters too.
#define ZP_KATTR_COLS __launch_bounds__(64 * ZP_WAVES)
// One streamed tile: descriptors given (len, ga), stream, walk, verdict,
// record store (the batch kernels).
template <bool COLS, bool TINY = !COLS, class L = WaveLds, bool SLOTS = false>
__device__ __forceinline__ void parse_tile(uint64_t t, uint32_t len, uintptr_t ga, uint64_t n,
                                           int lane, L& lds,
                                           zp_record* __restrict__ records,
                                           zp_ext_offsets* __restrict__ ext,
                                           const ColPtrs& cols) {
    const uintptr_t fallback = (uintptr_t)&zp_safe_chunk;   // dummy loads when T == 0
    uint4* win = &lds.win[0];
    uint4* tail = &lds.win[0] + ZP_WIN_CH * 64;
    // a tile of 64-B frames: registers only (wave-uniform test)
    if (TINY && !__ballot(t * 64 + lane < n && len != 64u) &&
        tiny_tile(t, len, ga, n, lane, records, SLOTS))
        return;
    TileState s;
    tile_setup(s, t, len, ga, n, lane, lds);
    // stream: one group of ZP_G items per iteration (group 0 outside the
    // loop, so no load is in flight across the loop back-edge)
    if (s.nitems <= ZP_SMALL_G) {              // wave-uniform: a tile of small frames
        // One group of ZP_SMALL_G items holds the whole tile (c2: 4 KiB):
        // no dummy loads past the tile's end (c2 -8 %, c5 -1 %, c3/c4 0).
        uint4 vs[ZP_SMALL_G];
        uint32_t ks[ZP_SMALL_G];
        issue_group<ZP_SMALL_G>(0, s.nitems, s.cur, s.R, lane, fallback, vs, ks);
        consume_group<ZP_SMALL_G>(0, s.nitems, lane, vs, ks, win, tail, lds.cend, s.run);
    } else
    {
    uint4 va[ZP_G];
    uint32_t ka[ZP_G];
    issue_group<ZP_G>(0, s.nitems, s.cur, s.R, lane, fallback, va, ka);
    consume_group<ZP_G>(0, s.nitems, lane, va, ka, win, tail, lds.cend, s.run);
    for (uint32_t i0 = ZP_G; i0 < s.nitems; i0 += ZP_G) {
        if (s.nitems - i0 <= 2) {                 // the last 1-2 items as a pair
            uint4 vt[2];
            uint32_t kt[2];
            issue_group<2>(i0, s.nitems, s.cur, s.R, lane, fallback, vt, kt);
            consume_group<2>(i0, s.nitems, lane, vt, kt, win, tail, lds.cend, s.run);
            break;
        }
        // The last <= ZP_TAIL_G items as a small group: fewer dummy loads
        // past the tile's end, whose address work (4 ds_bpermute each) and
        // consume are not free (c5 -1.7 %, c6 -1.1 %, c3 -0.3 %, c4 0;
        // profiles/r04_kbench_tail_group.log). Wave-uniform.
        if (s.nitems - i0 <= ZP_TAIL_G) {
            uint4 vt[ZP_TAIL_G];
            uint32_t kt[ZP_TAIL_G];
            issue_group<ZP_TAIL_G>(i0, s.nitems, s.cur, s.R, lane, fallback, vt, kt);
            consume_group<ZP_TAIL_G>(i0, s.nitems, lane, vt, kt, win, tail, lds.cend, s.run);
            break;
        }
        issue_group<ZP_G>(i0, s.nitems, s.cur, s.R, lane, fallback, va, ka);
        consume_group<ZP_G>(i0, s.nitems, lane, va, ka, win, tail, lds.cend, s.run);
    }
    }
    wave_lds_fence();                          // LDS written by other lanes
    // The frame address again, from its rank's stream origin (live
    // through the stream anyway) instead of keeping it there: two VGPRs
    // less at the stream's register peak. Only frames that own chunks
    // (>= 64 B) ever use it.
    {
        const uint32_t r = s.rank & 63u;
        const uintptr_t org = ((uintptr_t)bperm(s.R.org_hi, r) << 32) | bperm(s.R.org_lo, r);
        s.ga = org + 16ull * bperm(s.R.pfx, r) + s.shift;
    }
    __builtin_amdgcn_s_setprio(0);             // walk at priority 0 ...
    tile_finish<COLS, false, L, SLOTS>(s, n, lane, lds, records, ext, cols);
}

template <bool COLS, bool SLOTS = false>
__device__ __forceinline__ void parse_tiles(const uint8_t* __restrict__ arena,
                                            const uint64_t* __restrict__ offs,
                                            const uint32_t* __restrict__ lens, uint64_t n,
                                            zp_record* __restrict__ records,
                                            zp_ext_offsets* __restrict__ ext,
                                            const ColPtrs& cols) {
    __shared__ WaveLds lds_all[ZP_WAVES];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    WaveLds& lds = lds_all[wid];
    // ZP_K consecutive tiles per wave (one contiguous band of the arena)
    const uint64_t blk = blockIdx.x;
    for (uint32_t k = 0; k < ZP_K; ++k) {
        const uint64_t t = (blk * ZP_WAVES + wid) * ZP_K + k;
        if (t * 64 >= n) return;                   // wave-uniform
        // ... stream at priority 1: a streaming wave's load issue is not
        // queued behind a walking wave's VALU (c5 +1.8 %, c3/c4 +0-0.5 %)
        __builtin_amdgcn_s_setprio(1);
        if (k) wave_lds_fence();                   // previous tile's LDS reads done
        uint32_t len;
        uintptr_t ga;
        load_desc(arena, offs, lens, n, t, lane, len, ga);
        parse_tile<COLS, !COLS, WaveLds, SLOTS>(t, len, ga, n, lane, lds, records, ext, cols);
    }
}

#ifdef ZP_PARSE_SLOTS_TU
// The parse kernel with record slots, alone in its translation unit
// (zp_parse_slots.hip): compiled beside zp_parse_kernel in one module, the
// second instantiation of the tile code changed zp_parse_kernel's register
// allocation (2 VGPRs spilled, SGPRs 94 -> 98).
__global__ void ZP_KATTR
zp_parse_slots_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                      const uint32_t* __restrict__ lens, uint64_t n,
                      zp_record* __restrict__ records, zp_ext_offsets* __restrict__ ext) {
    const ColPtrs none{};
    parse_tiles<false, true>(arena, offs, lens, n, records, ext, none);
}
extern "C" __attribute__((visibility("hidden"))) hipError_t
zp__parse_slots_launch(uint64_t blocks, hipStream_t stream, const uint8_t* arena, const uint64_t* offs,
                       const uint32_t* lens, uint64_t n, zp_record* records, zp_ext_offsets* ext) {
    hipLaunchKernelGGL(zp_parse_slots_kernel, dim3((unsigned)blocks), dim3(64 * ZP_WAVES), 0, stream,
                       arena, offs, lens, n, records, ext);
    return hipGetLastError();
}
#else
extern "C" hipError_t zp__parse_slots_launch(uint64_t blocks, hipStream_t stream, const uint8_t* arena,
                                             const uint64_t* offs, const uint32_t* lens, uint64_t n,
                                             zp_record* records, zp_ext_offsets* ext);
__global__ void ZP_KATTR
zp_parse_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, uint64_t n,
                zp_record* __restrict__ records, zp_ext_offsets* __restrict__ ext) {
    const ColPtrs none{};
    parse_tiles<false>(arena, offs, lens, n, records, ext, none);
}

// The records of every code tile from its codes (after the parse kernel on
// the same stream): a wave takes ZP_EXPAND_TILES tiles, finds the code tiles
// among them from one byte each, and lane l rewrites record l of each from
// code l; a tile whose first bytes are a record is left as the parse stored
// it. Only full tiles can hold codes.
#define ZP_EXPAND_TILES 16    // tiles per wave: one load finds the code tiles among them
__global__ void __launch_bounds__(256) zp_rec_expand_kernel(zp_record* __restrict__ records, uint64_t n,
                                                             uint32_t* __restrict__ hint, uint32_t token) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t t0 = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * ZP_EXPAND_TILES;
    const uint64_t full = n / 64;                       // tiles that can hold codes
    // byte 3 of each tile (lanes 0-15): >= ZP_CODE_BASE marks a code tile
    const uint32_t b3 = lane < ZP_EXPAND_TILES && t0 + lane < full
                            ? ((const uint8_t*)(records + (t0 + lane) * 64))[3] : 0u;
    const uint64_t m = __ballot(b3 >= ZP_CODE_BASE);
    if (!m) return;
    // (a probe of the automatic mode: the first wave of every 64th
    // workgroup says, in mapped host memory, when at least 3/4 of its tiles
    // are code tiles: traffic with a few scattered code tiles, as config 5
    // has, stays on the one-kernel path)
    if (hint && lane == 0 && (threadIdx.x >> 6) == 0 && (blockIdx.x & 63u) == 0 &&
        __builtin_popcountll(m) * 4 >= 3 * ZP_EXPAND_TILES)
        __hip_atomic_store(hint, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t c[ZP_EXPAND_TILES];
#pragma unroll
    for (int k = 0; k < ZP_EXPAND_TILES; ++k)           // the codes, all loads in flight
        c[k] = (m >> k) & 1u ? ((const uint8_t*)(records + (t0 + k) * 64))[lane] : 0u;
#pragma unroll
    for (int k = 0; k < ZP_EXPAND_TILES; ++k)
        if ((m >> k) & 1u)
            __builtin_nontemporal_store(code_rec(c[k]), (zp_u32x2*)(records + (t0 + k) * 64 + lane));
}

extern "C" __attribute__((visibility("hidden"))) int zp__rec_expand_launch(zp_record* records, uint64_t n,
                                                                         hipStream_t stream,
                                                                         uint32_t* hint, uint32_t token) {
    if (n < 64) return 0;
    const uint64_t per_block = 4 * ZP_EXPAND_TILES;              // tiles
    hipLaunchKernelGGL(zp_rec_expand_kernel, dim3((unsigned)((n / 64 + per_block - 1) / per_block)),
                       dim3(256), 0, stream, records, n, hint, token);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_err("zp_rec_expand_kernel launch", e); return -2; }
    return 0;
}

// Record codes (0 auto: batches of at least ZP_SLOT_MIN_FRAMES, 1 always,
// 2 never): zp_set_record_slots. Below that the second launch costs more
// than the codes save (c2, 1M x 64 B).
#define ZP_SLOT_MIN_FRAMES (1ull << 21)
static int g_slot_mode = 0;
extern "C" int zp_set_record_slots(int mode) {
    if (mode < 0 || mode > 2) return -1;
    return __atomic_exchange_n(&g_slot_mode, mode, __ATOMIC_RELAXED);
}

// The automatic mode learns per device whether the traffic has code tiles:
// the first automatic call and every ZP_SLOT_PROBE_EVERY-th one after its
// predecessor's result is known run the code kernels with a mapped host
// word the expansion sets when sampled waves find mostly code tiles; once that call has
// completed (an event, queried without waiting) the following calls take
// the code kernels only if it found some. Traffic without code tiles (c5,
// c4) then runs zp_parse_kernel alone but for the probes. Under stream
// capture the last decision is used as is; a call with another batch size
// than the last probes at once. A hint only: either kernel writes the same
// records.
#define ZP_SLOT_PROBE_EVERY 16
struct SlotState {
    std::mutex mu;
    uint32_t* word = nullptr;          // mapped host word (host view)
    uint32_t* word_d = nullptr;        // its device view
    hipEvent_t ev = nullptr;
    bool pending = false, decision = true, broken = false;
    uint64_t since = 0;                // automatic calls since the last probe
    uint64_t last_n = 0;               // a new batch size probes at once
    uint32_t token = 0;                // the pending probe's (the word holds the last finder's)
};
static SlotState g_slot_state[64];

// The automatic mode's decision on the current device (1: the code kernels,
// 0: the one-kernel path), for reports.
extern "C" int zp_record_slots_state(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) { (void)hipGetLastError(); dev = 0; }
    SlotState& st = g_slot_state[dev & 63];
    std::lock_guard<std::mutex> guard(st.mu);
    return st.decision ? 1 : 0;
}

static bool slot_state_init(SlotState& st) {
    if (st.word || st.broken) return !st.broken;
    void* w = nullptr;
    if (hipHostMalloc(&w, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&st.word_d, w, 0) != hipSuccess ||
        hipEventCreateWithFlags(&st.ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        st.broken = true;                                    // decide without probes
        return false;
    }
    st.word = (uint32_t*)w;
    return true;
}

// Parse + column views in one pass (zp_parse_batch_columns_device).
__global__ void ZP_KATTR_COLS
zp_parse_columns_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                        const uint32_t* __restrict__ lens, uint64_t n,
                        zp_record* __restrict__ records, zp_ext_offsets* __restrict__ ext,
                        ColPtrs cols) {
    parse_tiles<true>(arena, offs, lens, n, records, ext, cols);
}

extern "C" int zp_parse_batch_device(const uint8_t* arena, const uint64_t* offs,
                                     const uint32_t* lens, uint64_t n,
                                     zp_record* records, zp_ext_offsets* ext,
                                     void* stream) {
    if (n == 0) return 0;
    if (!arena || !offs || !lens || !records) {
        snprintf(g_last_error, sizeof g_last_error, "zp_parse_batch_device: null pointer");
        return -1;
    }
    const uint64_t per_block = 64ull * ZP_WAVES * ZP_K;
    const uint64_t blocks = (n + per_block - 1) / per_block;
    if (blocks > 0x7FFFFFFFull) {
        snprintf(g_last_error, sizeof g_last_error, "zp_parse_batch_device: batch too large");
        return -1;
    }
    const int mode = __atomic_load_n(&g_slot_mode, __ATOMIC_RELAXED);
    const hipStream_t st_h = (hipStream_t)stream;
    auto launch = [&](bool slots, uint32_t* hint, uint32_t token) -> int {
        hipError_t e;
        if (slots) {
            e = zp__parse_slots_launch(blocks, st_h, arena, offs, lens, n, records, ext);
        } else {
            hipLaunchKernelGGL(zp_parse_kernel, dim3((unsigned)blocks), dim3(64 * ZP_WAVES), 0,
                               st_h, arena, offs, lens, n, records, ext);
            e = hipGetLastError();
        }
        if (e != hipSuccess) { set_err("zp_parse_kernel launch", e); return -2; }
        return slots ? zp__rec_expand_launch(records, n, st_h, hint, token) : 0;
    };
    if (mode != 0 || n < ZP_SLOT_MIN_FRAMES) return launch(mode == 1, nullptr, 0);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) { (void)hipGetLastError(); dev = 0; }
    SlotState& st = g_slot_state[dev & 63];
    std::lock_guard<std::mutex> guard(st.mu);
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st_h, &cs) != hipSuccess) { (void)hipGetLastError(); cs = hipStreamCaptureStatusActive; }
    if (cs != hipStreamCaptureStatusNone) return launch(st.decision, nullptr, 0);
    if (n != st.last_n) {                       // another workload: probe now
        st.last_n = n;
        st.since = 0;
        st.pending = false;                     // (a pending probe was the old workload's)
    }
    if (st.pending) {
        const hipError_t q = hipEventQuery(st.ev);
        if (q == hipSuccess) {
            st.decision = __atomic_load_n(st.word, __ATOMIC_ACQUIRE) == st.token;
            st.pending = false;
        } else {
            (void)hipGetLastError();                          // (hipErrorNotReady)
        }
    }
    if (st.pending || st.since++ % ZP_SLOT_PROBE_EVERY != 0 || !slot_state_init(st))
        return launch(st.decision, nullptr, 0);
    // a probe: its expansion writes this token when it finds code tiles (an
    // earlier probe still in flight writes its own)
    st.token = st.token + 1 ? st.token + 1 : 1;
    const int rc = launch(true, st.word_d, st.token);
    if (rc == 0 && hipEventRecord(st.ev, st_h) == hipSuccess) st.pending = true;
    else (void)hipGetLastError();
    return rc;
}

extern "C" int zp_parse_batch_columns_device(const uint8_t* arena, const uint64_t* offs,
                                             const uint32_t* lens, uint64_t n,
                                             zp_record* records, zp_ext_offsets* ext,
                                             void* const* cols, void* stream) {
    if (n == 0) return 0;
    if (!arena || !offs || !lens || !records || !cols) {
        snprintf(g_last_error, sizeof g_last_error, "zp_parse_batch_columns_device: null pointer");
        return -1;
    }
    ColPtrs c;
    for (int k = 0; k < ZP_COL_COUNT; ++k) c.p[k] = (uint8_t*)cols[k];
    const uint64_t per_block = 64ull * ZP_WAVES * ZP_K;
    const uint64_t blocks = (n + per_block - 1) / per_block;
    if (blocks > 0x7FFFFFFFull) {
        snprintf(g_last_error, sizeof g_last_error, "zp_parse_batch_columns_device: batch too large");
        return -1;
    }
    hipLaunchKernelGGL(zp_parse_columns_kernel, dim3((unsigned)blocks), dim3(64 * ZP_WAVES), 0,
                       (hipStream_t)stream, arena, offs, lens, n, records, ext, c);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_err("zp_parse_columns_kernel launch", e); return -2; }
    return 0;
}

// --------------------------------------------------------------------------
// zp_parse_one's resident server (zp_ctx.hip). PacketParser::parse for one
// frame (parser.rs:53) costs a kernel launch and its completion signal when
// each call launches the batch kernel (17.5 us). Instead one
// kernel per device stays resident, one wave per context slot, each polling
// a doorbell in its context's mapped host block: the host writes the frame,
// then the 64-bit doorbell (sequence << 32 | length); the wave sees it,
// parses the frame in place as a one-frame tile (the batch kernel's own
// tile_finish), writes the chains back into the block, and then the record,
// the sequence number and a tag in one 16-B store. The kernel leaves when it
// has been resident for `life` ticks of the 100 MHz constant clock
// (s_memrealtime; 1 ms by default, whatever the traffic) or when the retire
// word of the control block reaches its generation (the host queued the
// next generation behind it, or stops the server), so it never spins past
// use and a device-wide synchronisation waits for about one life at most.
// Memory order: the blocks are fine-grained (coherent) host memory. The
// doorbell, the retire word, the slot table and acknowledgement read at
// start and the frame bytes (stream
// and fallback loads) are read with system-scope loads (sc0 sc1, past both
// caches), so a frame the host rewrote since the last request is never
// served from a cache and no cache-wide invalidate is needed; the record and
// chain stores are system-scope (written through); the chain entries
// complete inside the tile, before the record store.
// --------------------------------------------------------------------------
#define ZP_ONE_BELL 0        // uint64_t: seq << 32 | frame length (host writes)
#define ZP_ONE_REC 64        // zp_record (server writes) ...
#define ZP_ONE_ACK 72        // ... and right after it, in the same 16-B store, the uint32_t
                             // seq of the last finished request
#define ZP_ONE_EXT 96        // zp_ext_offsets[2] (server writes)
#define ZP_ONE_FRAME 128     // the frame (host writes)
#define ZP_ONE_TAG 0x9E3779B9u    // answer tag: rec.x ^ rec.y ^ seq ^ ZP_ONE_TAG (zp_ctx.hip)
#define ZP_CTL_RETIRE 0      // control block (zp_ctx.hip SharedServer): uint32_t retire word
#define ZP_CTL_TABLE 64      // ... and uint64_t[64]: each slot's block

// The one frame of a zp_parse_one request, streamed by the server wave: its
// chunks [A & ~15, E) are contiguous, so lane l of item i simply loads chunk
// 64 i + l (system-scope; lanes past the frame load nothing), the first
// ZP_WIN_CH chunks go to the window cells of rank 0, the last to its tail
// cell, and the frame's word sum is one wave reduction per item. The batch
// stream's frame-start masks, rank permutes and running scans (tile_setup,
// issue_group, consume_group) have nothing to do here; the walk, verdict and
// record store are tile_finish's. Frames <= 64 KiB (ONE_MAX).
__device__ __forceinline__ void one_frame_tile(uint32_t len, uintptr_t ga, int lane, WaveLds& lds,
                                               zp_record* records, zp_ext_offsets* ext,
                                               uintptr_t sysbase, zp_u32x2* rec_out) {
    const ColPtrs none{};
    const uint32_t shift = (uint32_t)(ga & 15);
    const uint32_t nch = len >= 64 ? (len + shift + 15) >> 4 : 0u;   // as tile_setup
    const uintptr_t base = ga & ~(uintptr_t)15;
    uint32_t total = 0;
    for (uint32_t i0 = 0; i0 < nch; i0 += 64u * 4u) {
        uint4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t c = i0 + 64u * q + (uint32_t)lane;
            v[q] = ld_sys16(sysbase, c < nch ? base + 16ull * c : sysbase + 0xFFFFFFF0u);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t c = i0 + 64u * q + (uint32_t)lane;
            if (c < ZP_WIN_CH && c < nch) lds.win[c * 64 + c] = v[q];   // rank 0's cell c
            if (c + 1 == nch) lds.win[ZP_WIN_CH * 64] = v[q];            // rank 0's tail
            uint32_t part = sad16(v[q].x, 0u);
            part = sad16(v[q].y, part);
            part = sad16(v[q].z, part);
            part = sad16(v[q].w, part);
            total += rdl(wave_scan(c < nch ? part : 0u), 63);
        }
    }
    if (lane == 0) lds.cend[0] = total;
    wave_lds_fence();
    TileState s;
    s.tile = 0;
    s.ga = ga;
    s.live = lane == 0;
    s.len = lane == 0 ? len : 0u;
    s.shift = shift;
    s.wlen = s.len < ZP_WIN - shift ? s.len : ZP_WIN - shift;
    s.giant = false;
    s.rank = (uint32_t)lane;
    s.nitems = 0;
    s.run = 0;
    tile_finish<false, true>(s, 1, lane, lds, records, ext, none, sysbase, rec_out);
}

__global__ void __launch_bounds__(64)
zp_one_server_kernel(const uint8_t* ctl, uint64_t life, uint32_t gen) {
    __shared__ WaveLds lds;
    const int lane = threadIdx.x & 63;
    // This wave's slot: the block of one context (the table in the control
    // block, zp_ctx.hip SharedServer); an empty slot has nothing to serve.
    uint64_t b = 0;
    if (lane == 0)
        b = __hip_atomic_load((const uint64_t*)(ctl + ZP_CTL_TABLE) + blockIdx.x, __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_SYSTEM);
    uint8_t* blk = (uint8_t*)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(b >> 32), 0) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((uint32_t)b, 0));
    if (!blk) return;
    // The last answered request is the slot's acknowledgement word (the
    // previous generation's, or the host's after a give-up): a wave never
    // answers a request twice, and answers one rung while it waited for the
    // stream.
    uint32_t seq = 0;
    if (lane == 0)
        seq = __hip_atomic_load((const uint32_t*)(blk + ZP_ONE_ACK), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_SYSTEM);
    seq = (uint32_t)__builtin_amdgcn_readlane(seq, 0);
    // One system-scope poll of the doorbell in flight, from lane 0 (loads of
    // one address from several lanes are not merged and cost ~0.1 us each),
    // and of the retire word from lane 1, in one load instruction. Measured
    // and not kept (profiles/r05_parse_one_server_iterations.log): four
    // polling waves per slot (7.2 us per call: they slow the working wave's
    // host accesses), and several polls in flight from this wave (the
    // compiler waits for all of them at the rotation's head).
    // The kernel leaves once it has been resident for `life` ticks, or at
    // once when the retire word reaches its generation (the host queued the
    // next one behind it or stops the server): a device-wide synchronisation
    // issued meanwhile (hipDeviceSynchronize, torch.cuda.synchronize,
    // hipFree) waits about that long at most.
    const uint64_t born = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        uint64_t bell = 0;
        if (lane < 2)
            bell = __hip_atomic_load(lane ? (const uint64_t*)(ctl + ZP_CTL_RETIRE)
                                          : (const uint64_t*)(blk + ZP_ONE_BELL),
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t bseq = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(bell >> 32), 0);
        const uint32_t blen = (uint32_t)__builtin_amdgcn_readlane((uint32_t)bell, 0);
        const uint32_t retire = (uint32_t)__builtin_amdgcn_readlane((uint32_t)bell, 1);
        if ((int32_t)(retire - gen) >= 0) break;             // a newer generation / a stop
        if (bseq == seq) {
            if (__builtin_amdgcn_s_memrealtime() - born > life) break;
            __builtin_amdgcn_s_sleep(1);                     // ~64 clocks between polls
            continue;
        }
        seq = bseq;
        {                                                    // a request (wave-uniform)
            __builtin_amdgcn_s_setprio(1);
            // every load of the frame and every store of the results is
            // system-scope (SYS): nothing is left in a cache to invalidate
            // or write back
            zp_u32x2 rec{0u, 0u};
            one_frame_tile(blen, (uintptr_t)(blk + ZP_ONE_FRAME), lane, lds,
                           (zp_record*)(blk + ZP_ONE_REC), (zp_ext_offsets*)(blk + ZP_ONE_EXT),
                           (uintptr_t)blk, &rec);
            // The record and the acknowledgement in one 16-B store, so
            // nothing waits for the record's completion first (a host-link
            // round trip, ~1.2 us; the chain entries, when there are any,
            // completed inside the tile). The fourth word tags the record
            // with the seq (ZP_ONE_TAG): the host accepts the answer only
            // when ack and tag agree with the record it read, so a 16-B
            // write the host link delivered in pieces is waited out, not
            // returned.
            if (lane == 0)
                st_sys16((uintptr_t)blk, (uintptr_t)(blk + ZP_ONE_REC),
                         zp_u32x4{rec.x, rec.y, bseq, rec.x ^ rec.y ^ bseq ^ ZP_ONE_TAG});
            wave_lds_fence();                                 // LDS reused by the next request
            __builtin_amdgcn_s_setprio(0);                    // polls at the base priority
            if (__builtin_amdgcn_s_memrealtime() - born > life) break;
        }
    }
}

extern "C" __attribute__((visibility("hidden"))) int zp__one_server_launch(const uint8_t* ctl_d,
                                                                            uint32_t nslots,
                                                                            uint64_t life_ticks,
                                                                            uint32_t gen,
                                                                            void* stream) {
    if (nslots == 0) return 0;
    hipLaunchKernelGGL(zp_one_server_kernel, dim3(nslots), dim3(64), 0, (hipStream_t)stream, ctl_d,
                       life_ticks, gen);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_err("zp_one_server_kernel launch", e); return -2; }
    return 0;
}

// Test hook (zp__one_test_hooks, zp_ctx.hip): one wave that spins for `ticks`
// of the constant clock, queued in front of a server launch to make the
// server start late.
__global__ void __launch_bounds__(64) zp_one_stall_kernel(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

extern "C" __attribute__((visibility("hidden"))) int zp__one_stall_launch(uint64_t ticks,
                                                                           void* stream) {
    hipLaunchKernelGGL(zp_one_stall_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ticks);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_err("zp_one_stall_kernel launch", e); return -2; }
    return 0;
}
#endif  // ZP_PARSE_SLOTS_TU
