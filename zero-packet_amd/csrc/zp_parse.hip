// zp_parse.hip — MI355X (gfx950) batched PacketParser::parse.
//
// Reference path: /root/reference/src/packet/parser.rs:53-140 (parse,
// parse_ipv4, parse_ipv6, parse_protocol) with the readers it calls
// (ethernet.rs:141-212, arp.rs:130-176, ipv4.rs:138-264, ipv6.rs:147-285,
// extensions/headers.rs:51-213, tcp.rs:141-213, udp.rs:103-135,
// icmpv4.rs:92-104, icmpv6.rs:89-101) and the checksum primitives
// (checksum.rs:5-69).
//
// Kernel structure (one 256-thread workgroup = one tile of 256 frames):
//   A. cooperative window load: the first 128 B of every frame of the tile
//      (16-B aligned chunks, 8 consecutive lanes per frame -> coalesced) into
//      an LDS window stored dword-column-major: win[dword][frame], so a lane
//      reading ANY dword of its own frame hits bank (frame % 32): no conflicts.
//   B. lane-per-frame header walk from LDS (global byte loads only for bytes
//      past the window): Ethernet/VLAN -> ARP / IPv4 / IPv6 + extension chain
//      -> IP-in-IP levels -> TCP/UDP/ICMP checks, IPv4 header checksums, the
//      pseudo-header sum and the L4 bytes that sit inside the window.
//   C. flattened stream: the remaining L4 bytes of all frames of the tile form
//      a list of 16-B aligned chunks (exclusive scan of per-frame chunk
//      counts); lane k of the workgroup loads chunk k, k+256, ... so each wave
//      reads 1 KiB of mostly contiguous arena per load. A wave-wide prefix sum
//      plus run boundaries turns per-chunk sums into per-frame sums, added to
//      LDS accumulators once per (frame, 1 KiB block).
//   D. finalize: checksum validity from the exact partial sums, record store.
//
// Checksum arithmetic. The reference verifies S = acc + sum of big-endian
// 16-bit words (u32), valid iff !fold(S) as u16 == 0 (checksum.rs:5-35),
// i.e. S != 0 and S == 0 (mod 65535). We sum little-endian 16-bit words at
// even ARENA addresses (V = E + 256*O, E/O = sums of bytes at even/odd
// addresses) because that is what aligned dword loads give for free:
//   segment starting at an odd address:  W = V exactly,
//   segment starting at an even address: W == 256*V (mod 65535),
// and W == 0 iff V == 0. Exact u32 sums hold for segments <= 64 KiB; longer
// (IPv6 jumbo) segments take an exact E/O path that reproduces the
// reference's u32 wrap-around.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/zero_packet.h"
#include "zp_errstr.h"

#define ZP_TILE 256          // frames per workgroup (= threads)
#define ZP_WIN 128           // window bytes per frame
#define ZP_WIN_DW (ZP_WIN / 4)
#define ZP_WIN_CH (ZP_WIN / 16)
#define ZP_GIANT 65536u      // segments longer than this take the exact path
#define ZP_UNROLL 4          // stream blocks in flight per wave

static __thread char g_last_error[256];

static void set_err(const char* what, hipError_t e) {
    snprintf(g_last_error, sizeof g_last_error, "%s: %s", what, hipGetErrorString(e));
}

extern "C" const char* zp_last_error(void) { return g_last_error; }
extern "C" __attribute__((visibility("hidden"))) char* zp__errbuf(void) { return g_last_error; }
extern "C" int zp_abi_version(void) { return ZP_ABI_VERSION; }
extern "C" const char* zp_err_str(int code) { return zp_err_string(code); }

// --------------------------------------------------------------------------
// Device helpers
// --------------------------------------------------------------------------

// Valid ICMPv4 types (misc.rs:93-119) / ICMPv6 types (misc.rs:164-204) as
// 256-bit sets.
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

// Checksum validity from the arena-parity sum V of a segment starting at an
// address of parity `odd`, with accumulator acc (fast path, exact V).
__device__ __forceinline__ bool csum_ok(uint32_t acc, uint32_t V, bool odd) {
    if (acc == 0 && V == 0) return false;                  // S == 0 -> 0xFFFF
    uint32_t w = V % 65535u;
    if (!odd) w = (w * 256u) % 65535u;
    return ((acc % 65535u) + w) % 65535u == 0;
}

// View of one frame: LDS window column + global fallback.
struct FrameView {
    const uint32_t* col;     // &win[0][slot]; dword d at col[d * ZP_TILE]
    const uint8_t* g;        // frame in global memory
    uint32_t shift;          // frame address & 15 (window starts 16-aligned)
    uint32_t wlen;           // frame bytes available in the window
    uint32_t len;            // frame length
};

__device__ __forceinline__ uint32_t rd8(const FrameView& f, uint32_t x) {
    if (x < f.wlen) {
        uint32_t y = x + f.shift;
        return (f.col[(y >> 2) * ZP_TILE] >> ((y & 3) * 8)) & 0xFFu;
    }
    return f.g[x];
}
__device__ __forceinline__ uint32_t rd16(const FrameView& f, uint32_t x) {
    return (rd8(f, x) << 8) | rd8(f, x + 1);
}

// Arena-parity word sum V of frame bytes [lo, hi) (both <= len).
__device__ uint32_t sumV(const FrameView& f, uint32_t lo, uint32_t hi) {
    uint32_t s = 0;
    uint32_t h1 = hi < f.wlen ? hi : f.wlen;
    if (lo < h1) {
        int ylo = (int)(lo + f.shift), yhi = (int)(h1 + f.shift);
        for (int d = ylo >> 2; d <= (yhi - 1) >> 2; ++d)
            s = sad16(f.col[d * ZP_TILE] & byte_mask(d * 4, ylo, yhi), s);
    }
    uint32_t l2 = lo > f.wlen ? lo : f.wlen;
    if (l2 < hi) {
        uintptr_t a0 = (uintptr_t)f.g + l2, a1 = (uintptr_t)f.g + hi;
        for (uintptr_t d = a0 & ~(uintptr_t)3; d < a1; d += 4) {
            uint32_t v = *(const uint32_t*)d;
            s = sad16(v & byte_mask(0, (int)((intptr_t)a0 - (intptr_t)d),
                                    (int)((intptr_t)a1 - (intptr_t)d)), s);
        }
    }
    return s;
}

// Exact reference checksum for long segments: sums even/odd-address bytes
// separately and reproduces the u32 wrap of checksum.rs:12 (release build).
__device__ bool csum_ok_exact(const uint8_t* g, uint32_t lo, uint32_t hi, uint32_t acc) {
    uint64_t E = 0, O = 0;
    uintptr_t a0 = (uintptr_t)g + lo, a1 = (uintptr_t)g + hi;
    for (uintptr_t d = a0 & ~(uintptr_t)3; d < a1; d += 4) {
        uint32_t v = *(const uint32_t*)d;
        v &= byte_mask(0, (int)((intptr_t)a0 - (intptr_t)d), (int)((intptr_t)a1 - (intptr_t)d));
        E += (v & 0xFFu) + ((v >> 16) & 0xFFu);
        O += ((v >> 8) & 0xFFu) + (v >> 24);
    }
    uint64_t W = (a0 & 1) ? (256ull * O + E) : (256ull * E + O);
    uint32_t S = (uint32_t)(acc + W);
    while (S >> 16) S = (S & 0xFFFFu) + (S >> 16);
    return (uint16_t)~S == 0;
}

// Per-frame walk result.
struct Walk {
    zp_record rec;
    zp_ext_offsets inner;
    uint32_t acc;        // pseudo-header accumulator of the innermost IP
    uint32_t l4;         // L4 start (frame offset) when a checksum is pending
    uint8_t pending;     // 1 = L4 checksum still to verify
    uint8_t v6;          // innermost IP is IPv6 (selects the error code)
};

// Extension-header walk (headers.rs:51-213). Returns 0 or a zp_err.
// pos = IPv6 payload start; outputs slot offsets relative to pos.
__device__ int ext_walk(const FrameView& f, uint32_t pos, uint32_t nh,
                        uint32_t* present, uint16_t off[6], uint32_t* total,
                        uint32_t* final_nh) {
    uint32_t pres = 0, tot = 0, fin = 0;
    uint32_t cur = nh, p = pos;
    for (int it = 0; it < 8; ++it) {
        uint32_t rem = f.len - p;
        int slot;
        uint32_t hl;
        if (cur == 0) {                                   // Hop-by-Hop (:90-113)
            if (pres & 1) break;
            if (pres) return ZP_ERR_EXT_HBH_NOT_FIRST;
            if (rem < 8) return ZP_ERR_EXT_OPTIONS_TOO_SHORT;
            hl = (rd8(f, p + 1) + 1) * 8;
            if (hl > rem) return ZP_ERR_EXT_OPTIONS_EXCEEDS;
            slot = ZP_EXT_HBH;
        } else if (cur == 43) {                           // Routing (:117-134)
            if (pres & 2) break;
            if (rem < 8) return ZP_ERR_EXT_ROUTING_TOO_SHORT;
            hl = (rd8(f, p + 1) + 1) * 8;
            if (hl > rem) return ZP_ERR_EXT_ROUTING_EXCEEDS;
            slot = ZP_EXT_RT;
        } else if (cur == 44) {                           // Fragment (:138-155)
            if (pres & 4) break;
            if (rem < 8) return ZP_ERR_EXT_FRAGMENT_TOO_SHORT;
            hl = 8;
            slot = ZP_EXT_FRAG;
        } else if (cur == 51) {                           // Authentication (:159-176)
            if (pres & 8) break;
            if (rem < 12) return ZP_ERR_EXT_AUTH_TOO_SHORT;
            hl = (rd8(f, p + 1) + 2) * 4;
            if (hl > rem) return ZP_ERR_EXT_AUTH_EXCEEDS;
            slot = ZP_EXT_AH;
        } else if (cur == 60) {                           // Destination (:180-202)
            if (pres & 32) break;
            if (rem < 8) return ZP_ERR_EXT_OPTIONS_TOO_SHORT;
            hl = (rd8(f, p + 1) + 1) * 8;
            if (hl > rem) return ZP_ERR_EXT_OPTIONS_EXCEEDS;
            slot = (pres & 16) ? ZP_EXT_DST2 : ZP_EXT_DST1;
        } else {
            break;
        }
        uint32_t next = rd8(f, p);
        pres |= 1u << slot;
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if (k == slot) off[k] = (uint16_t)(p - pos);   // constant index: stays in VGPRs
        tot += hl;
        fin = next;
        cur = next;
        p += hl;
    }
    *present = pres;
    *total = tot;
    *final_nh = fin;
    return 0;
}

// The header-chain walk of PacketParser::parse for one frame.
__device__ void walk_frame(const FrameView& f, Walk& w) {
    zp_record& r = w.rec;
    w.pending = 0; w.acc = 0; w.l4 = 0; w.v6 = 0;
    const uint32_t len = f.len;
    int err = 0;
    if (len < 64) { err = ZP_ERR_ETH_FRAME_TOO_SHORT; goto done; }   // parser.rs:159
    {
        uint32_t hl = 14;                                             // ethernet.rs:155-179
        uint32_t t0 = rd16(f, 12);
        if (t0 == 0x8100) hl = 18;
        else if (t0 == 0x88A8) {
            if (rd16(f, 16) != 0x8100) { err = ZP_ERR_ETH_INVALID_QINQ; goto done; }
            hl = 22;
        }
        r.eth_len = (uint8_t)hl;
        uint32_t et = rd16(f, hl - 2);                                 // ethernet.rs:209-212
        if (et == 0x0806) {                                           // ARP, parser.rs:60,172-180
            if (len - hl < 28) { err = ZP_ERR_ARP_TOO_SHORT; goto done; }
            if (rd16(f, hl + 6) > 2) { err = ZP_ERR_ARP_INVALID_OPER; goto done; }
            r.flags |= ZP_F_ARP;
        } else if (et == 0x0800 || et == 0x86DD) {
            uint32_t pos = hl;
            bool v4 = et == 0x0800;
            for (uint32_t level = 0;; ++level) {
                uint32_t sl = len - pos;                              // slice length
                uint32_t proto, pp, acc;
                if (v4) {                                             // parser.rs:188-212
                    if (sl < 20) { err = ZP_ERR_IPV4_TOO_SHORT; goto done; }
                    uint32_t b0 = rd8(f, pos);
                    if ((b0 >> 4) != 4) { err = ZP_ERR_IPV4_VERSION; goto done; }
                    uint32_t ihl = (b0 & 15) * 4;
                    if (ihl < 20) { err = ZP_ERR_IPV4_IHL_TOO_SHORT; goto done; }
                    if (sl < ihl) { err = ZP_ERR_IPV4_HDR_TOO_LONG; goto done; }
                    if (rd16(f, pos + 2) != sl) { err = ZP_ERR_IPV4_TOTAL_LENGTH; goto done; }
                    uint32_t hv = sumV(f, pos, pos + ihl);             // ipv4.rs:262-264
                    if (!(hv != 0 && hv % 65535u == 0)) { err = ZP_ERR_IPV4_CHECKSUM; goto done; }
                    proto = rd8(f, pos + 9);
                    pp = pos + ihl;
                    if (proto == 1) acc = 0;                          // parser.rs:322-326
                    else acc = rd16(f, pos + 12) + rd16(f, pos + 14) + rd16(f, pos + 16) +
                               rd16(f, pos + 18) + proto + (len - pp);
                    if (level == 0) r.flags |= ZP_F_IPV4;
                    else if (level == 1) { r.flags |= ZP_F_IP_IN_IP; r.inner_off = pos; }
                } else {                                              // parser.rs:222-230
                    if (sl < 40) { err = ZP_ERR_IPV6_TOO_SHORT; goto done; }
                    uint32_t pres = 0, tot = 0, fin = 0;
                    uint16_t eo[6] = {0, 0, 0, 0, 0, 0};
                    uint32_t nh = rd8(f, pos + 6);
                    int e = ext_walk(f, pos + 40, nh, &pres, eo, &tot, &fin);   // ipv6.rs:159
                    if (e) { err = e; goto done; }
                    if ((rd8(f, pos) >> 4) != 6) { err = ZP_ERR_IPV6_VERSION; goto done; }
                    proto = pres ? fin : nh;                          // ipv6.rs:219-227
                    pp = pos + 40 + tot;                              // ipv6.rs:283-285
                    acc = proto + (len - pp);                         // parser.rs:349-354
                    for (uint32_t k = 0; k < 32; k += 2) acc += rd16(f, pos + 8 + k);
                    if (level == 0) {
                        r.flags |= ZP_F_IPV6;
                        r.final_nh = (uint8_t)proto;
                        if (pres) {
                            r.flags |= ZP_F_EXT | (pres << 12);
                            r.ext_len = (uint16_t)tot;
                            for (int k = 0; k < 6; ++k) r.ext_off[k] = eo[k];
                        }
                    } else if (level == 1) {
                        r.flags |= ZP_F_IP_IN_IP | ZP_F_IP_IN_IP_V6;
                        r.inner_off = pos;
                        r.inner_final_nh = (uint8_t)proto;
                        if (pres) {
                            r.flags |= ZP_F_INNER_EXT | (pres << 18);
                            r.inner_ext_len = (uint16_t)tot;
                            for (int k = 0; k < 6; ++k) w.inner.off[k] = eo[k];
                        }
                    }
                }
                uint32_t rem = len - pp;                              // parse_protocol :111-140
                if (proto == 6) {
                    if (rem < 20) { err = ZP_ERR_TCP_TOO_SHORT; goto done; }
                    if ((rd8(f, pp + 12) >> 4) * 4 < 20) { err = ZP_ERR_TCP_DATA_OFFSET; goto done; }
                    if (rd8(f, pp + 13) == 0) { err = ZP_ERR_TCP_FLAGS; goto done; }
                    r.flags |= ZP_F_TCP;
                } else if (proto == 17) {
                    if (rem < 8) { err = ZP_ERR_UDP_TOO_SHORT; goto done; }
                    if (rd16(f, pp + 4) != rem) { err = ZP_ERR_UDP_LENGTH; goto done; }
                    r.flags |= ZP_F_UDP;
                } else if (proto == 1) {
                    if (rem < 8) { err = ZP_ERR_ICMP_TOO_SHORT; goto done; }
                    if (!icmpv4_type_ok(rd8(f, pp))) { err = ZP_ERR_ICMPV4_TYPE; goto done; }
                    if (rd8(f, pp + 1) > 15) { err = ZP_ERR_ICMPV4_CODE; goto done; }
                    r.flags |= ZP_F_ICMPV4;
                } else if (proto == 58) {
                    if (rem < 8) { err = ZP_ERR_ICMP_TOO_SHORT; goto done; }
                    if (!icmpv6_type_ok(rd8(f, pp))) { err = ZP_ERR_ICMPV6_TYPE; goto done; }
                    r.flags |= ZP_F_ICMPV6;
                } else if (proto == 4 || proto == 41) {               // IP-in-IP recursion
                    v4 = proto == 4;
                    pos = pp;
                    continue;
                } else {
                    break;                                            // unknown: Ok, no L4
                }
                r.l4_off = pp;
                w.pending = 1;
                w.acc = acc;
                w.l4 = pp;
                w.v6 = v4 ? 0 : 1;
                break;
            }
        }
        r.flags |= ZP_F_ETHERNET;
    }
done:
    if (err) {
        r = zp_record{};
        r.err = (uint8_t)err;
        w.pending = 0;
    }
}

// --------------------------------------------------------------------------
// The batch kernel.
// --------------------------------------------------------------------------
struct __align__(16) TileShared {
    uint32_t win[ZP_WIN_DW][ZP_TILE];   // 32 KiB, dword-column-major windows
    uint64_t seg_base[ZP_TILE];         // 16-aligned address of the first stream chunk
    uint32_t seg_lo[ZP_TILE];           // first valid byte in the first chunk
    uint32_t seg_hi[ZP_TILE];           // end byte relative to seg_base
    uint32_t pre[ZP_TILE + 1];          // exclusive scan of chunk counts
    uint32_t acc[ZP_TILE];              // streamed V partial sums
    uint32_t wsum[ZP_TILE / 64];
};

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__global__ void __launch_bounds__(ZP_TILE)
zp_parse_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, uint64_t n,
                zp_record* __restrict__ records, zp_ext_offsets* __restrict__ inner_ext) {
    __shared__ TileShared sh;
    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wid = t >> 6;
    const uint64_t p0 = (uint64_t)blockIdx.x * ZP_TILE;
    const uint64_t p = p0 + t;
    const bool live = p < n;

    // ---- descriptors
    uint64_t off = live ? offs[p] : 0;
    uint32_t len = live ? lens[p] : 0;
    const uint8_t* g = arena + off;

    // ---- A. cooperative window load: item j -> frame j / 8, chunk j % 8.
    // Descriptors go through LDS (seg_base / seg_hi are free until phase C).
    sh.seg_base[t] = (uint64_t)(uintptr_t)g;
    sh.seg_hi[t] = len;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < ZP_WIN_CH; ++k) {
        int j = k * ZP_TILE + t;
        int fr = j / ZP_WIN_CH, ch = j % ZP_WIN_CH;
        {
            uint32_t fl = sh.seg_hi[fr];                  // 0 for frames past n
            uintptr_t fa = (uintptr_t)sh.seg_base[fr];
            uintptr_t ca = (fa & ~(uintptr_t)15) + 16u * ch;
            if (fl >= 64 && ca < fa + fl) {
                uint4 v = *(const uint4*)ca;
                sh.win[ch * 4 + 0][fr] = v.x;
                sh.win[ch * 4 + 1][fr] = v.y;
                sh.win[ch * 4 + 2][fr] = v.z;
                sh.win[ch * 4 + 3][fr] = v.w;
            }
        }
    }
    __syncthreads();

    // ---- B. walk
    FrameView fv;
    fv.col = &sh.win[0][t];
    fv.g = g;
    fv.shift = (uint32_t)((uintptr_t)g & 15);
    fv.len = len;
    {
        uint32_t avail = ZP_WIN - fv.shift;
        fv.wlen = len < avail ? len : avail;
    }
    Walk w;
    w.rec = zp_record{};
    w.inner = zp_ext_offsets{};
    if (live) walk_frame(fv, w);
    else w.pending = 0;

    // Checksum job: window part now, stream part [S, len) later.
    uint32_t vwin = 0, nchunks = 0;
    bool giant = false;
    if (w.pending) {
        if (len - w.l4 > ZP_GIANT) {
            giant = true;
        } else {
            uint32_t wend = len < fv.wlen ? len : fv.wlen;
            if (w.l4 < wend) vwin = sumV(fv, w.l4, wend);
            uint32_t S = w.l4 > fv.wlen ? w.l4 : fv.wlen;
            if (S < len) {
                uintptr_t sa = (uintptr_t)g + S, ea = (uintptr_t)g + len;
                uintptr_t base = sa & ~(uintptr_t)15;
                nchunks = (uint32_t)((ea - base + 15) >> 4);
                sh.seg_base[t] = base;
                sh.seg_lo[t] = (uint32_t)(sa - base);
                sh.seg_hi[t] = (uint32_t)(ea - base);
            }
        }
    }
    sh.acc[t] = 0;

    // Block exclusive scan of chunk counts.
    uint32_t inc = wave_incl_scan(nchunks, lane);
    if (lane == 63) sh.wsum[wid] = inc;
    __syncthreads();
    uint32_t wbase = 0, total = 0;
#pragma unroll
    for (int k = 0; k < ZP_TILE / 64; ++k) {
        uint32_t s = sh.wsum[k];
        wbase += k < wid ? s : 0;
        total += s;
    }
    sh.pre[t] = wbase + inc - nchunks;
    if (t == 0) sh.pre[ZP_TILE] = total;
    __syncthreads();

    // ---- C. flattened stream over all pending chunks of the tile.
    {
        uint32_t cur = 0;   // segment cursor (wave-uniform)
        for (uint32_t blk0 = (uint32_t)wid * 64; blk0 < total; blk0 += ZP_TILE * ZP_UNROLL) {
            uint4 v[ZP_UNROLL];
            int seg[ZP_UNROLL];
            uint32_t lo[ZP_UNROLL], hi[ZP_UNROLL];
#pragma unroll
            for (int u = 0; u < ZP_UNROLL; ++u) {
                uint32_t kb = blk0 + u * ZP_TILE;       // block start item
                uint32_t k = kb + lane;
                seg[u] = -1;
                v[u] = make_uint4(0, 0, 0, 0);
                if (kb < total) {
                    while (sh.pre[cur + 1] <= kb) ++cur;          // first segment of block
                    int s = cur;
                    for (int q = cur; q < ZP_TILE && sh.pre[q] < kb + 64; ++q)
                        if (k >= sh.pre[q]) s = q;
                    if (k < total) {
                        seg[u] = s;
                        uint32_t i = k - sh.pre[s];
                        lo[u] = sh.seg_lo[s];
                        hi[u] = sh.seg_hi[s];
                        lo[u] = lo[u] > 16u * i ? lo[u] - 16u * i : 0u;
                        hi[u] = hi[u] - 16u * i;          // > 0 for a valid item
                        v[u] = *(const uint4*)(sh.seg_base[s] + 16ull * i);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < ZP_UNROLL; ++u) {
                uint32_t kb = blk0 + u * ZP_TILE;
                if (kb >= total) break;
                uint32_t s16 = 0;
                if (seg[u] >= 0) {
                    int l = (int)lo[u], h = hi[u] > 16u ? 16 : (int)hi[u];
                    if (l == 0 && h == 16) {
                        s16 = sad16(v[u].x, s16);
                        s16 = sad16(v[u].y, s16);
                        s16 = sad16(v[u].z, s16);
                        s16 = sad16(v[u].w, s16);
                    } else {
                        s16 = sad16(v[u].x & byte_mask(0, l, h), s16);
                        s16 = sad16(v[u].y & byte_mask(4, l, h), s16);
                        s16 = sad16(v[u].z & byte_mask(8, l, h), s16);
                        s16 = sad16(v[u].w & byte_mask(12, l, h), s16);
                    }
                }
                // Segmented reduction: prefix sum + run boundaries.
                uint32_t ps = wave_incl_scan(s16, lane);
                int sprev = __shfl_up(seg[u], 1, 64);
                int snext = __shfl_down(seg[u], 1, 64);
                bool first = lane == 0 || sprev != seg[u];
                bool last = lane == 63 || snext != seg[u];
                uint64_t firsts = __ballot(first);
                // run start lane for this lane
                uint64_t below = firsts & ((lane == 63) ? ~0ull : ((2ull << lane) - 1ull));
                int start = 63 - __builtin_clzll(below);
                uint32_t before = __shfl(ps, start > 0 ? start - 1 : 0, 64);
                if (start == 0) before = 0;
                if (last && seg[u] >= 0) atomicAdd(&sh.acc[seg[u]], ps - before);
            }
        }
    }
    __syncthreads();

    // ---- D. finalize + store
    if (!live) return;
    zp_record r = w.rec;
    if (w.pending) {
        bool ok;
        if (giant) {
            ok = csum_ok_exact(g, w.l4, len, w.acc);
        } else {
            uint32_t V = vwin + sh.acc[t];
            bool odd = ((uintptr_t)(g + w.l4)) & 1;
            ok = csum_ok(w.acc, V, odd);
        }
        if (!ok) {
            r = zp_record{};
            r.err = (uint8_t)(w.v6 ? ZP_ERR_IPV6_L4_CHECKSUM : ZP_ERR_IPV4_L4_CHECKSUM);
        }
    }
    uint4 q[2];
    memcpy(q, &r, sizeof r);
    uint4* dst = (uint4*)(records + p);
    dst[0] = q[0];
    dst[1] = q[1];
    if (inner_ext && (r.flags & ZP_F_INNER_EXT)) inner_ext[p] = w.inner;
}

// --------------------------------------------------------------------------
// C ABI
// --------------------------------------------------------------------------
extern "C" int zp_parse_batch_device(const uint8_t* arena, const uint64_t* offs,
                                     const uint32_t* lens, uint64_t n,
                                     zp_record* records, zp_ext_offsets* inner_ext,
                                     void* stream) {
    if (n == 0) return 0;
    if (!arena || !offs || !lens || !records) {
        snprintf(g_last_error, sizeof g_last_error, "zp_parse_batch_device: null pointer");
        return -1;
    }
    uint64_t blocks = (n + ZP_TILE - 1) / ZP_TILE;
    if (blocks > 0x7FFFFFFFull) {
        snprintf(g_last_error, sizeof g_last_error, "zp_parse_batch_device: batch too large");
        return -1;
    }
    hipLaunchKernelGGL(zp_parse_kernel, dim3((unsigned)blocks), dim3(ZP_TILE), 0,
                       (hipStream_t)stream, arena, offs, lens, n, records, inner_ext);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_err("zp_parse_kernel launch", e); return -2; }
    return 0;
}
