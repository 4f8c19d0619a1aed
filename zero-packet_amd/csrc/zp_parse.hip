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

#define ZP_WIN 128           // window bytes per frame
#define ZP_WIN_DW (ZP_WIN / 4)
#define ZP_WIN_CH (ZP_WIN / 16)
#define ZP_GIANT 65536u      // segments longer than this take the exact path
// Timing-only ablations (tools/build_variants.sh); never set in the product:
//   ZP_ABL_WIN_OFF   skip the window load
//   ZP_ABL_FAKE_WALK replace the walk by "pending L4 at offset 42"
//   ZP_ABL_STREAM_OFF skip the stream loads

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
    const uint32_t* col;     // &win[wave][0][0]; see win_dw()
    uint32_t lane;
    const uint8_t* g;        // frame in global memory
    uint32_t shift;          // frame address & 15 (window starts 16-aligned)
    uint32_t wlen;           // frame bytes available in the window
    uint32_t len;            // frame length
};

// Window dword d of frame `lane` lives at win[d][lane ^ 4*(d/4)]: the XOR
// keeps both the cooperative chunk writes (8 frames x 8 chunks per
// instruction) and the per-lane reads conflict-free.
__device__ __forceinline__ uint32_t win_dw(const FrameView& f, uint32_t d) {
    return f.col[d * 64 + (f.lane ^ ((d >> 2) << 2))];
}

__device__ __forceinline__ uint32_t rd8(const FrameView& f, uint32_t x) {
    if (x < f.wlen) {
        uint32_t y = x + f.shift;
        return (win_dw(f, y >> 2) >> ((y & 3) * 8)) & 0xFFu;
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
            s = sad16(win_dw(f, d) & byte_mask(d * 4, ylo, yhi), s);
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
// The batch kernel. Every wave is independent: it owns 64 consecutive frames
// (lane j = frame j), so no workgroup barrier is ever needed; a workgroup is
// just 4 waves packed for occupancy.
// --------------------------------------------------------------------------

// Wave-wide sum with DPP (row_shr 1/2/4/8 + row_bcast 15/31 inclusive scan,
// lane 63 holds the total); returns the wave-uniform total.
__device__ __forceinline__ uint32_t wave_total(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ uint32_t rdl(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

typedef unsigned zp_u32x4 __attribute__((ext_vector_type(4)));

// Streamed 16-B chunk, read once: nontemporal.
__device__ __forceinline__ uint4 ld_stream(uintptr_t a) {
    zp_u32x4 v = __builtin_nontemporal_load((const zp_u32x4*)a);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// V-sum of bytes [l, h) of a 16-B chunk (l in [0,16), h in (0,16]).
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

#define ZP_WAVES 4
#ifndef ZP_G
#define ZP_G 4        // stream items per group; two groups in flight per wave
#endif

// One stream item = (frame j of the wave, 1 KiB block k of its stream range).
struct Items {
    int j[ZP_G];
    uint32_t k[ZP_G];
};

// Stream state of a wave: frames with blocks left in the current pass.
struct Cursor {
    uint64_t mask;
    uint32_t pass;
    bool done;
};

__device__ __forceinline__ void fill_items(Items& it, Cursor& cur, uint32_t nblk) {
#pragma unroll
    for (int q = 0; q < ZP_G; ++q) {
        if (!cur.done && cur.mask == 0) {
            ++cur.pass;
            cur.mask = __ballot(nblk > cur.pass);
            cur.done = cur.mask == 0;
        }
        if (!cur.done) {
            it.j[q] = __builtin_ctzll(cur.mask);
            it.k[q] = cur.pass;
            cur.mask &= cur.mask - 1;
        } else {
            it.j[q] = -1;
            it.k[q] = 0;
        }
    }
}

// Issues the loads of a group: lane l reads chunk 64k + l of frame j.
__device__ __forceinline__ void issue_items(const Items& it, uint4 (&v)[ZP_G], int lane,
                                            uint32_t sb_lo, uint32_t sb_hi, uint32_t nch) {
#pragma unroll
    for (int q = 0; q < ZP_G; ++q) {
        v[q] = make_uint4(0, 0, 0, 0);
        if (it.j[q] >= 0) {
            const int j = it.j[q];
            const uint32_t c = it.k[q] * 64u + (uint32_t)lane;
            const uintptr_t b = ((uintptr_t)rdl(sb_hi, j) << 32) | rdl(sb_lo, j);
#ifndef ZP_ABL_STREAM_OFF
            if (c < rdl(nch, j)) v[q] = ld_stream(b + 16ull * c);
#endif
        }
    }
}

// Sums a landed group (full chunks only; lanes past the frame hold zeros)
// and adds each item's total to its frame's lane.
__device__ __forceinline__ void process_items(const Items& it, const uint4 (&v)[ZP_G], int lane,
                                              uint32_t& vsum) {
#pragma unroll
    for (int q = 0; q < ZP_G; ++q) {
        if (it.j[q] < 0) break;
        uint32_t part = sad16(v[q].x, 0u);
        part = sad16(v[q].y, part);
        part = sad16(v[q].z, part);
        part = sad16(v[q].w, part);
        const uint32_t tot = wave_total(part);
        if (lane == it.j[q]) vsum += tot;
    }
}

#ifdef ZP_MINW
__global__ void __launch_bounds__(64 * ZP_WAVES, ZP_MINW)
#else
__global__ void __launch_bounds__(64 * ZP_WAVES)
#endif
zp_parse_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, uint64_t n,
                zp_record* __restrict__ records, zp_ext_offsets* __restrict__ inner_ext) {
    // Per-wave LDS windows, dword-column-major: win[wave][dword][frame].
    __shared__ uint32_t win[ZP_WAVES][ZP_WIN_DW][64];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const uint64_t f0 = ((uint64_t)blockIdx.x * ZP_WAVES + wid) * 64;
    if (f0 >= n) return;                       // whole wave past the batch (uniform)
    const uint64_t p = f0 + lane;
    const bool live = p < n;
    const uint32_t len = live ? lens[p] : 0;
    const uint8_t* g = arena + (live ? offs[p] : 0);
    const uintptr_t ga = (uintptr_t)g;
    uint32_t* wcol = &win[wid][0][0];

    // ---- A. window load: instruction k covers frames 8k..8k+7, 8 lanes each
    // (128 contiguous bytes per frame), registers -> LDS columns.
#ifndef ZP_ABL_WIN_OFF
    {
        const uint32_t alo = (uint32_t)ga, ahi = (uint32_t)(ga >> 32);
#pragma unroll
        for (int k = 0; k < ZP_WIN_CH; ++k) {
            const int fr = k * 8 + (lane >> 3), ch = lane & 7;
            const uint32_t fl = __shfl(len, fr, 64);
            const uintptr_t fa = ((uintptr_t)(uint32_t)__shfl(ahi, fr, 64) << 32) |
                                 (uint32_t)__shfl(alo, fr, 64);
            const uintptr_t ca = (fa & ~(uintptr_t)15) + 16u * ch;
            if (fl >= 64 && ca < fa + fl) {
                uint4 v = *(const uint4*)ca;
                const int col = fr ^ (ch << 2);
                wcol[(ch * 4 + 0) * 64 + col] = v.x;
                wcol[(ch * 4 + 1) * 64 + col] = v.y;
                wcol[(ch * 4 + 2) * 64 + col] = v.z;
                wcol[(ch * 4 + 3) * 64 + col] = v.w;
            }
        }
    }
#endif

    // ---- Stream range, fixed BEFORE the walk. Past the window the frame is
    // 16-B aligned (the window ends at its 16-aligned base + 128), so the
    // stream is the full chunks [wend, ea & ~15); the partial tail chunk is
    // summed by the frame's own lane. Frames of 64 B..64 KiB only; the walk
    // later corrects for an L4 start on either side of the window end.
    const uint32_t shift = (uint32_t)(ga & 15);
    const uint32_t wlen = len < ZP_WIN - shift ? len : ZP_WIN - shift;
    const bool giant = len > ZP_GIANT;
    uint32_t nch = 0;
    uintptr_t sbase = 0;
    uint4 tail = make_uint4(0, 0, 0, 0);
    uint32_t tail_n = 0;                     // valid bytes in the tail chunk
    if (len >= 64 && !giant && wlen < len) {
        const uintptr_t ea = ga + len;
        sbase = ga + wlen;                   // 16-aligned
        nch = (uint32_t)(((ea & ~(uintptr_t)15) - sbase) >> 4);
        tail_n = (uint32_t)(ea & 15);
        if (tail_n) tail = *(const uint4*)(ea & ~(uintptr_t)15);
    }
    const uint32_t nblk = (nch + 63) >> 6;
    const uint32_t sb_lo = (uint32_t)sbase, sb_hi = (uint32_t)(sbase >> 32);
    Cursor cur;
    cur.mask = __ballot(nblk > 0);
    cur.pass = 0;
    cur.done = cur.mask == 0;
    Items ia, ib;
    uint4 va[ZP_G], vb[ZP_G];
    fill_items(ia, cur, nblk);
    issue_items(ia, va, lane, sb_lo, sb_hi, nch);      // in flight during the walk

    // LDS written by other lanes of this wave: order the wave's LDS ops.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- B. walk (lane per frame)
    FrameView fv;
    fv.col = wcol;
    fv.lane = (uint32_t)lane;
    fv.g = g;
    fv.shift = shift;
    fv.len = len;
    fv.wlen = wlen;
    Walk w;
    w.rec = zp_record{};
    w.inner = zp_ext_offsets{};
#ifdef ZP_ABL_FAKE_WALK
    w.pending = live && len >= 64;
    w.l4 = 42; w.acc = 0; w.v6 = 0;
    w.rec.flags = ZP_F_ETHERNET;
#else
    if (live) walk_frame(fv, w);
    else w.pending = 0;
#endif
    // L4 bytes inside the window and in the tail chunk, minus header bytes
    // the stream covers.
    uint32_t vsum = 0, vsub = 0;
    if (w.pending && !giant) {
        if (w.l4 < wlen) vsum = sumV(fv, w.l4, wlen);
        else if (w.l4 > wlen) vsub = sumV(fv, wlen, w.l4);
        if (tail_n) vsum = chunk_sum(tail, 0, (int)tail_n, vsum);
    }

    // ---- C. stream: two groups of ZP_G items in flight (ping-pong).
    while (ia.j[0] >= 0) {
        fill_items(ib, cur, nblk);
        issue_items(ib, vb, lane, sb_lo, sb_hi, nch);
        process_items(ia, va, lane, vsum);
        if (ib.j[0] < 0) break;
        fill_items(ia, cur, nblk);
        issue_items(ia, va, lane, sb_lo, sb_hi, nch);
        process_items(ib, vb, lane, vsum);
    }

    // ---- D. finalize + store
    if (!live) return;
    zp_record r = w.rec;
    if (w.pending) {
        bool ok;
        if (giant) {
            ok = csum_ok_exact(g, w.l4, len, w.acc);
        } else {
            bool odd = (ga + w.l4) & 1;
            ok = csum_ok(w.acc, vsum - vsub, odd);
        }
        if (!ok) {
            r = zp_record{};
            r.err = (uint8_t)(w.v6 ? ZP_ERR_IPV6_L4_CHECKSUM : ZP_ERR_IPV4_L4_CHECKSUM);
        }
    }
    uint4 q2[2];
    memcpy(q2, &r, sizeof r);
    uint4* dst = (uint4*)(records + p);
    dst[0] = q2[0];
    dst[1] = q2[1];
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
    uint64_t blocks = (n + 64 * ZP_WAVES - 1) / (64 * ZP_WAVES);
    if (blocks > 0x7FFFFFFFull) {
        snprintf(g_last_error, sizeof g_last_error, "zp_parse_batch_device: batch too large");
        return -1;
    }
    hipLaunchKernelGGL(zp_parse_kernel, dim3((unsigned)blocks), dim3(64 * ZP_WAVES), 0,
                       (hipStream_t)stream, arena, offs, lens, n, records, inner_ext);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { set_err("zp_parse_kernel launch", e); return -2; }
    return 0;
}
