// zp_build.hip — batched PacketBuilder.
//
// Reference: builder.rs:55-909 (the typestate chain) and the writers it
// calls: EthernetWriter ethernet.rs:19-129, ArpWriter arp.rs:7-119,
// IPv4Writer ipv4.rs:8-127, IPv6Writer ipv6.rs:8-133, Options/Routing/
// Fragment/AuthenticationHeaderWriter (extensions/*.rs), TcpWriter
// tcp.rs:7-130, UdpWriter udp.rs:7-92, Icmpv4Writer icmpv4.rs:10-81,
// Icmpv6Writer icmpv6.rs:7-78; checksums checksum.rs:5-69.
//
// One group of ZB_G lanes per frame, 64 / ZB_G frames per wave side by side:
// a chain is a serial program (every lane of the group runs it), its payload
// copy and the L4 checksum over the rest of the buffer are group-wide work.
// Frames up to ZB_CAP bytes (+ alignment) are staged in LDS with the chain's
// ops in one round trip: the group executes the chain on the LDS copy and
// writes back only the bytes the chain can have changed. Longer frames run
// in place in global memory, every lane of the group on the same bytes.
//
// The chain's scalar steps run on every lane with identical values (every
// lane stores the same byte to the same address), so each lane reads back
// its own writes and no cross-lane ordering is needed except after the
// cooperative steps (staging, copies), which end with a wave barrier.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/zero_packet.h"
#include "zp_stream.h"

extern "C" char* zp__errbuf(void);

#define ZB_WAVES 4
#define ZB_CAP 1536            // frame bytes staged in LDS per frame
#define ZB_LDS (ZB_CAP + 32)   // + the frame's offset in its first 16-B chunk
#define ZB_OPS 4               // ops of a chain prefetched to LDS (longer chains read the rest)
#define ZB_WPE 4               // waves per SIMD: 128 VGPRs (5 spilled at 96: 13 % slower on
#define ZB_G 16                // lanes per frame: a wave builds 64 / ZB_G frames side by side
#define ZB_F (64 / ZB_G)       // frames per wave
#define ZB_PENDING 0xFFu       // results[i].err: left by the lane path for the lane-group pass

// Exact reference strings (see zero_packet.h for the cited lines).
static const char* const kBuildErr[ZP_BERR_COUNT] = {
    "",
    "Slice is too short to contain an Ethernet frame.",
    "Slice is too short to contain VLAN tagging.",
    "Slice is too short to contain double VLAN tagging.",
    "Data too short to contain an ARP header.",
    "Slice is too short to contain an ARP header.",
    "Data too short to contain an IPv4 header.",
    "Slice is too short to contain an IPv4 header.",
    "Data too short to contain an IPv6 header.",
    "Slice is too short to contain an IPv6 header.",
    "Data too short to contain a TCP segment.",
    "Slice is too short to contain a TCP header.",
    "Payload is too large to fit in the TCP packet.",
    "Data too short to contain a UDP datagram.",
    "Slice is too short to contain a UDP header.",
    "Data too short to contain an ICMP packet.",
    "Slice is too short to contain an ICMP header.",
    "Payload is too large to fit in the ICMPv4 packet.",
    "Data too short to contain an ICMPv6 packet.",
    "Payload is too large to fit in the ICMPv6 packet.",
    "Data too short to contain an IPv6 Hop-by-Hop Options header.",
    "Data too short to contain an IPv6 Destination Options header.",
    "Slice is too short to contain an Options extension header.",
    "Options field must be at least 6 bytes long.",
    "Options length must match the header extension length.",
    "Options exceed the allocated header length.",
    "Data too short to contain an IPv6 Routing header.",
    "Slice is too short to contain a Routing extension header.",
    "Type-specific data must be at least 4 bytes long.",
    "Type-specific data length must match the header extension length.",
    "Type-specific data exceeds the allocated header length.",
    "Data too short to contain an IPv6 Authentication header.",
    "Slice is too short to contain an Authentication extension header.",
    "Authentication data exceeds the allocated header length.",
    "panic (the reference builder would panic here)",
    "invalid builder chain (does not type-check against builder.rs:817-909)",
};

extern "C" const char* zp_build_err_str(int code) {
    return code >= 0 && code < ZP_BERR_COUNT ? kBuildErr[code] : nullptr;
}

// Builder typestates (builder.rs:29-45).
enum { BS_RAW, BS_ETH, BS_ARP, BS_V4, BS_V6, BS_HBH, BS_D1, BS_RT, BS_FR, BS_AH, BS_D2, BS_V4E,
       BS_V6E, BS_L4 };

// builder.rs:817-909: the state reached by method `k` from state `st`, -1 if
// the chain would not compile.
__device__ __forceinline__ int bnext(int st, int k) {
    const bool l4v4 = k == ZP_B_TCP || k == ZP_B_UDP || k == ZP_B_ICMPV4;
    const bool l4v6 = k == ZP_B_TCP || k == ZP_B_UDP || k == ZP_B_ICMPV6;
    switch (st) {
    case BS_RAW: return (k >= ZP_B_ETHERNET && k <= ZP_B_ETHERNET_QINQ) ? BS_ETH : -1;
    case BS_ETH: return k == ZP_B_ARP ? BS_ARP : k == ZP_B_IPV4 ? BS_V4 : k == ZP_B_IPV6 ? BS_V6 : -1;
    case BS_V4: return l4v4 ? BS_L4 : k == ZP_B_IPV4 ? BS_V4E : k == ZP_B_IPV6 ? BS_V6E : -1;
    case BS_V4E: return l4v4 ? BS_L4 : -1;
    case BS_V6E: return l4v6 ? BS_L4 : -1;
    case BS_V6: case BS_HBH: case BS_D1: case BS_RT: case BS_FR: case BS_AH: case BS_D2: {
        if (l4v6) return BS_L4;
        if (k == ZP_B_IPV4) return BS_V4E;
        if (k == ZP_B_IPV6) return BS_V6E;
        // extension header order (RFC 2460, builder.rs:850-909): each state's
        // permitted successors as a mask over {HBH, D1, RT, FR, AH, D2}
        const uint32_t succ[7] = {0x3F, 0x3E, 0x04, 0x38, 0x30, 0x20, 0x00};
        const int e = k == ZP_B_HOP_BY_HOP ? 0 : k == ZP_B_DEST_OPTS1 ? 1 : k == ZP_B_ROUTING ? 2
                    : k == ZP_B_FRAGMENT ? 3 : k == ZP_B_AUTH ? 4 : k == ZP_B_DEST_OPTS2 ? 5 : -1;
        if (e < 0 || !((succ[st - BS_V6] >> e) & 1)) return -1;
        return BS_HBH + e;
    }
    default: return -1;
    }
}

// Frame view for the chain. Every lane executes the chain's stores with the
// same values and reads back its own stores: no cross-lane dependency through
// memory outside the cooperative steps, which end in wave_sync(). (Stores by
// lane 0 alone read by the other lanes would be a data race: the compiler may
// forward a lane's earlier load past another lane's store.)
// LDS mode (P = LDS pointer): copies and the checksum are lane-strided.
// Global mode (P = generic pointer to the frame in place, frames past the
// LDS size): every lane runs everything on the same bytes.
#define ZB_LDSP __attribute__((address_space(3)))
typedef unsigned zb_u32x4 __attribute__((ext_vector_type(4)));

template <typename P>
struct BView {
    P b;
    uint32_t n;
    bool writer;      // this lane stores
    uint32_t lim = ~0u;   // ZB_M_WIN: blob copies stop at this frame offset (the rest: HBM)
};

template <typename P>
__device__ __forceinline__ void w8(BView<P>& v, uint32_t i, uint32_t x) {
    if (v.writer) v.b[i] = (uint8_t)x;
}
template <typename P>
__device__ __forceinline__ void w16(BView<P>& v, uint32_t i, uint32_t x) {
    w8(v, i, x >> 8);
    w8(v, i + 1, x);
}
template <typename P>
__device__ __forceinline__ void w32(BView<P>& v, uint32_t i, uint32_t x) {
    w16(v, i, x >> 16);
    w16(v, i + 2, x);
}
template <typename P>
__device__ __forceinline__ void wbytes(BView<P>& v, uint32_t i, const uint8_t* s, int k) {
#pragma unroll
    for (int q = 0; q < k; ++q) w8(v, i + q, s[q]);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Execution modes of a chain: ZB_M_COOP — a lane group on an LDS copy of
// the frame; ZB_M_GLOBAL — a lane group in place in global memory (long
// frames); ZB_M_WIN — one lane on its frame's window in the packed-stream
// LDS layout (the lane-per-frame path, zp_build_fast_kernel).
enum { ZB_M_COOP = 0, ZB_M_GLOBAL = 1, ZB_M_WIN = 2 };


// Copies `len` bytes of the data blob to frame offset `at`.
template <int MODE, typename P>
__device__ void bcopy(BView<P>& v, uint32_t at, const uint8_t* src, uint32_t len, int lane,
                      bool payload = false) {
    if constexpr (MODE == ZB_M_COOP) {
        // Aligned dword loads of the blob (address space 1: they cannot alias
        // the LDS stores, so four are in flight per lane), byte stores to the
        // staged frame. One byte per lane and trip was 20 % slower on
        // payload-copy chains (tools/build_bench.py --payload).
        const uintptr_t sa = (uintptr_t)src, sb = sa & ~(uintptr_t)3;
        const uint32_t sh = (uint32_t)(sa & 3);
        const ZP_GLOBAL uint32_t* g32 = (const ZP_GLOBAL uint32_t*)sb;
        for (uint32_t k0 = lane; 4 * k0 < len; k0 += 4 * ZB_G) {
            uint32_t d[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t k = k0 + u * ZB_G;
                uint32_t lo = 0, hi = 0;
                if (4 * k < len) {
                    lo = g32[k];
                    if (sh && sb + 4 * (k + 1) < sa + len) hi = g32[k + 1];
                }
                d[u] = __builtin_amdgcn_alignbyte(hi, lo, sh);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t k = k0 + u * ZB_G;
#pragma unroll
                for (uint32_t b = 0; b < 4; ++b)
                    if (4 * k + b < len) v.b[at + 4 * k + b] = (uint8_t)(d[u] >> (8 * b));
            }
        }
        wave_sync();
    } else if constexpr (MODE == ZB_M_WIN) {
        // the part inside the lane's window; a payload past it goes to HBM
        // after the chain (zp_build_fast_kernel)
        // (only the final payload copy is cut: extension data lies inside
        // the chain's extent, which the window holds)
        const uint32_t lim = payload ? v.lim : ~0u;
        const uint32_t m = at >= lim ? 0u : (lim - at < len ? lim - at : len);
        for (uint32_t q = 0; q < m; ++q) v.b[at + q] = src[q];
    } else {
        for (uint32_t q = 0; q < len; ++q) v.b[at + q] = src[q];
    }
}

// S = acc + sum of big-endian words of bytes[s0 .. n) (checksum.rs:11-20; a
// trailing odd byte counts as its high byte), folded and inverted
// (checksum.rs:23-28). Exact: the word sum is 256 * (bytes at even positions
// from s0) + (bytes at odd positions), both plain byte sums.
// LDS mode: `stage` is the wave's staging buffer and `shift` the frame's
// offset in it; each lane sums whole 16-B cells with v_sad_u8 over
// even/odd-address byte masks, then a wave reduction.
__device__ uint16_t bcsum_lds(const uint8_t ZB_LDSP* stage, uint32_t shift, uint32_t s0,
                              uint32_t n, uint32_t acc, int lane) {
    const uint32_t p0 = shift + s0, p1 = shift + n;      // staged byte range
    uint32_t ev = 0, od = 0;                             // bytes at even / odd staged positions
    for (uint32_t c = (p0 >> 4) + lane; 16 * c < p1; c += ZB_G) {
        const zb_u32x4 q = *(const zb_u32x4 ZB_LDSP*)(stage + 16 * c);
        const uint32_t d[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int base = (int)(16 * c + 4 * k);
            const int lo = (int)p0 - base, hi = (int)p1 - base;
            const uint32_t a = lo < 0 ? 0u : (lo > 4 ? 4u : (uint32_t)lo);
            const uint32_t b = hi < 0 ? 0u : (hi > 4 ? 4u : (uint32_t)hi);
            const uint32_t m = (uint32_t)(0xFFFFFFFFull >> (32 - 8 * b)) &
                               ~(uint32_t)(0xFFFFFFFFull >> (32 - 8 * a));
            const uint32_t x = d[k] & m;
            ev = __builtin_amdgcn_sad_u8(x & 0x00FF00FFu, 0u, ev);
            od = __builtin_amdgcn_sad_u8(x & 0xFF00FF00u, 0u, od);
        }
    }
#pragma unroll
    for (int off = ZB_G / 2; off > 0; off >>= 1) {     // within the frame's lane group
        ev += (uint32_t)__shfl_xor((int)ev, off);
        od += (uint32_t)__shfl_xor((int)od, off);
    }
    uint32_t sum = acc + ((p0 & 1) ? 256u * od + ev : 256u * ev + od);
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t)~sum;
}

// Global mode: the reference's sequential loop (u32 wrap included).
__device__ uint16_t bcsum_seq(const uint8_t* b, uint32_t s0, uint32_t n, uint32_t acc) {
    uint32_t sum = acc;
    uint32_t i = s0;
    for (; i + 1 < n; i += 2) sum += ((uint32_t)b[i] << 8) | b[i + 1];
    if (i < n) sum += (uint32_t)b[i] << 8;
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t)~sum;
}

// checksum.rs:43-69 over 4- or 16-byte addresses (constant indices only).
__device__ __forceinline__ uint32_t pseudo(const zp_build_op& o, bool v4, uint32_t proto,
                                           uint32_t length) {
    uint32_t s4 = 0, s16 = 0;
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        const uint32_t w = (((uint32_t)o.src[k] << 8) | o.src[k + 1]) +
                           (((uint32_t)o.dst[k] << 8) | o.dst[k + 1]);
        s16 += w;
        if (k < 4) s4 += w;
    }
    return (v4 ? s4 : s16) + proto + length;
}

// Op k of the chain: the first ZB_OPS from the wave's LDS copy (fetched with
// the frame in one round trip), the rest from global memory.
struct OpSrc {
    const zp_build_op ZB_LDSP* lds;
    const zp_build_op* g;
    __device__ __forceinline__ zp_build_op get(uint32_t k) const {
        if (k < ZB_OPS) {
            zp_build_op o;
            const zb_u32x4 ZB_LDSP* q = (const zb_u32x4 ZB_LDSP*)(lds + k);
            zb_u32x4 t[4] = {q[0], q[1], q[2], q[3]};
            __builtin_memcpy(&o, t, sizeof o);
            return o;
        }
        return g[k];
    }
    __device__ __forceinline__ uint32_t kind(uint32_t k) const {
        return k < ZB_OPS ? lds[k].kind : g[k].kind;
    }
};

struct NoWin {
    __device__ uint16_t csum(uint32_t, uint32_t) const { return 0; }
};

// Executes one chain (all checks of the reference, in its order). Returns
// the zp_build_err; *hl_out = header_len after the last Ok op, *hw_out = an
// upper bound of the bytes written ([0, hw)).
template <int MODE, typename P, typename OPS, typename WC>
__device__ __forceinline__ int run_chain(BView<P>& v, const uint8_t ZB_LDSP* stage, uint32_t shift,
                         const OPS& ops, uint32_t nops, const WC& wc,
                         const uint8_t* __restrict__ data, int lane, uint32_t* hl_out,
                         uint32_t* done_out, uint32_t* hw_out, uint32_t* doff_out = nullptr,
                         uint32_t* kind_out = nullptr) {
    int st = BS_RAW;
    *hw_out = 0;
    for (uint32_t k = 0; k < nops; ++k) {            // typestate (compile time in Rust)
        st = bnext(st, (int)ops.kind(k));
        if (st < 0) { *hl_out = 0; *done_out = 0; return ZP_BERR_TRANSITION; }
    }
    st = BS_RAW;
    uint32_t hl = 0, hw = 0;
    const uint32_t n = v.n;
    for (uint32_t k = 0; k < nops; ++k) {
        const zp_build_op o = ops.get(k);
        const int prev = st;
        st = bnext(st, o.kind);
        const bool has = o.data_len != ZP_BUILD_NO_DATA;
        const uint32_t dl = has ? o.data_len : 0u;
        const uint8_t* d = data + o.data_off;
        if (doff_out) *doff_out = o.data_off;        // the last op's, for the copy past the window
        if (kind_out) *kind_out = o.kind;
        const uint32_t sl = n - hl;                  // &mut bytes[header_len..]
        const uint32_t base = hl;
        P s = v.b + hl;
        uint32_t ext = 0;                            // bytes this op may write from `base`
        int e = 0;
        switch (o.kind) {
        case ZP_B_ETHERNET: case ZP_B_ETHERNET_VLAN: case ZP_B_ETHERNET_QINQ: {
            ext = 22;
            if (n < 14) { e = ZP_BERR_ETH_SLICE; break; }               // ethernet.rs:29-31
            wbytes(v, 6, o.src, 6);                                      // set_src_mac
            wbytes(v, 0, o.dst, 6);                                      // set_dest_mac
            uint32_t h = 14;
            if (o.kind == ZP_B_ETHERNET_VLAN) {                          // set_vlan_tag :83-96
                if (n < h + 4) { e = ZP_BERR_ETH_VLAN; break; }
                w16(v, 12, 0x8100); w16(v, 14, o.h[1]);
                h += 4;
            } else if (o.kind == ZP_B_ETHERNET_QINQ) {                   // :104-128
                if (n < h + 8) { e = ZP_BERR_ETH_QINQ; break; }
                w16(v, 12, 0x88A8); w16(v, 14, o.h[1]);
                w16(v, 16, 0x8100); w16(v, 18, o.h[2]);
                h += 8;
            }
            w16(v, 12 + (h - 14), o.h[0]);                               // set_ethertype
            hl = h;
            break;
        }
        case ZP_B_ARP:                                                   // builder.rs:203-236
            ext = 28;
            if (n < hl) { e = ZP_BERR_ARP_DATA; break; }
            if (sl < 28) { e = ZP_BERR_ARP_SLICE; break; }
            w16(v, hl, o.h[0]); w16(v, hl + 2, o.h[1]); w8(v, hl + 4, o.b[0]); w8(v, hl + 5, o.b[1]);
            w16(v, hl + 6, o.h[2]);
            wbytes(v, hl + 8, o.src, 6); wbytes(v, hl + 14, o.src + 6, 4);
            wbytes(v, hl + 18, o.dst, 6); wbytes(v, hl + 24, o.dst + 6, 4);
            hl += 28;
            break;
        case ZP_B_IPV4: {                                                // builder.rs:248-292
            ext = 20;
            if (n < hl) { e = ZP_BERR_IPV4_DATA; break; }
            if (sl < 20) { e = ZP_BERR_IPV4_SLICE; break; }
            w8(v, hl, (s[0] & 0x0F) | (uint8_t)(o.b[0] << 4));          // ipv4.rs:33-72
            w8(v, hl, (s[0] & 0xF0) | (o.b[1] & 0x0F));
            w8(v, hl + 1, (s[1] & 0x03) | (uint8_t)(o.b[2] << 2));
            w8(v, hl + 1, (s[1] & 0xFC) | (o.b[3] & 0x03));
            w16(v, hl + 2, o.h[0]);
            w16(v, hl + 4, o.h[1]);
            w8(v, hl + 6, (s[6] & 0x1F) | ((uint8_t)(o.b[4] << 5) & 0xE0));
            w8(v, hl + 6, (s[6] & 0xE0) | ((o.h[2] >> 8) & 0x1F));
            w8(v, hl + 7, o.h[2] & 0xFF);
            w8(v, hl + 8, o.b[5]);
            w8(v, hl + 9, o.b[6]);
            wbytes(v, hl + 12, o.src, 4);
            wbytes(v, hl + 16, o.dst, 4);
            const uint32_t ihl = (uint32_t)(s[0] & 0x0F) * 4;           // set_checksum :119-126
            w8(v, hl + 10, 0); w8(v, hl + 11, 0);
            if (ihl > sl) { e = ZP_BERR_PANIC; break; }                  // &bytes[..header_len]
            uint32_t sum = 0;
            for (uint32_t q = 0; q + 1 < ihl; q += 2) sum += ((uint32_t)s[q] << 8) | s[q + 1];
            while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
            w16(v, hl + 10, (uint16_t)~sum);
            hl += ihl;
            break;
        }
        case ZP_B_IPV6:                                                  // builder.rs:300-335
            ext = 40;
            if (n < hl) { e = ZP_BERR_IPV6_DATA; break; }
            if (sl < 40) { e = ZP_BERR_IPV6_SLICE; break; }
            w8(v, hl, (s[0] & 0x0F) | (uint8_t)(o.b[0] << 4));          // ipv6.rs:33-61
            w8(v, hl, (s[0] & 0xF0) | (o.b[1] >> 4));
            w8(v, hl + 1, (s[1] & 0x0F) | (uint8_t)(o.b[1] << 4));
            w8(v, hl + 1, (s[1] & 0xF0) | (uint8_t)(o.w[0] >> 16));     // unmasked, as :49
            w8(v, hl + 2, o.w[0] >> 8);
            w8(v, hl + 3, o.w[0]);
            w16(v, hl + 4, o.h[0]);
            w8(v, hl + 6, o.b[2]);
            w8(v, hl + 7, o.b[3]);
            wbytes(v, hl + 8, o.src, 16);
            wbytes(v, hl + 24, o.dst, 16);
            hl += 40;
            break;
        case ZP_B_HOP_BY_HOP: case ZP_B_DEST_OPTS1: case ZP_B_DEST_OPTS2: // builder.rs:611-806
            ext = 2 + dl;
            if (n < hl) { e = o.kind == ZP_B_HOP_BY_HOP ? ZP_BERR_HBH_DATA : ZP_BERR_DEST_DATA; break; }
            if (sl < 8) { e = ZP_BERR_OPTIONS_SLICE; break; }
            w8(v, hl, o.b[0]);
            w8(v, hl + 1, o.b[1]);
            if (dl < 6) { e = ZP_BERR_OPTIONS_MIN; break; }             // options.rs:53-68
            if ((uint32_t)s[1] * 8 != dl) { e = ZP_BERR_OPTIONS_MATCH; break; }
            if (2 + dl > sl) { e = ZP_BERR_OPTIONS_EXCEED; break; }
            bcopy<MODE>(v, hl + 2, d, dl, lane);
            hl += ((uint32_t)s[1] + 1) * 8;
            break;
        case ZP_B_ROUTING:                                               // builder.rs:675-704
            ext = 8 + dl;
            if (n < hl) { e = ZP_BERR_ROUTING_DATA; break; }
            if (sl < 8) { e = ZP_BERR_ROUTING_SLICE; break; }
            w8(v, hl, o.b[0]); w8(v, hl + 1, o.b[1]); w8(v, hl + 2, o.b[2]); w8(v, hl + 3, o.b[3]);
            if (dl < 4) { e = ZP_BERR_ROUTING_MIN; break; }             // routing.rs:75-94
            if ((uint32_t)s[1] * 8 != dl) { e = ZP_BERR_ROUTING_MATCH; break; }
            if (8 + dl > sl) { e = ZP_BERR_ROUTING_EXCEED; break; }
            bcopy<MODE>(v, hl + 8, d, dl, lane);
            hl += ((uint32_t)s[1] + 1) * 8;
            break;
        case ZP_B_FRAGMENT: {                                            // builder.rs:711-740
            ext = 8;
            if (n < hl) { e = ZP_BERR_ROUTING_DATA; break; }            // (its message)
            if (sl < 8) { e = ZP_BERR_PANIC; break; }                   // fragment.rs:15-17
            w8(v, hl, o.b[0]);
            w8(v, hl + 1, 0);
            const uint32_t fo = o.h[0] & 0x1FFF;                        // fragment.rs:52-80
            w8(v, hl + 2, fo >> 5);
            w8(v, hl + 3, (s[3] & 0xE0) | (fo & 0x1F));
            w8(v, hl + 3, s[3] & 0x9F);
            w8(v, hl + 3, o.b[1] ? (s[3] | 0x80) : (s[3] & 0x7F));
            w32(v, hl + 4, o.w[0]);
            hl += 8;
            break;
        }
        case ZP_B_AUTH:                                                  // builder.rs:747-778
            ext = 12 + dl;
            if (n < hl) { e = ZP_BERR_AUTH_DATA; break; }
            if (sl < 12) { e = ZP_BERR_AUTH_SLICE; break; }
            w8(v, hl, o.b[0]); w8(v, hl + 1, o.b[1]); w8(v, hl + 2, 0); w8(v, hl + 3, 0);
            w32(v, hl + 4, o.w[0]);
            w32(v, hl + 8, o.w[1]);
            if (12 + dl > sl) { e = ZP_BERR_AUTH_EXCEED; break; }       // authentication.rs:84-92
            bcopy<MODE>(v, hl + 12, d, dl, lane);
            hl += ((uint32_t)s[1] + 2) * 4;
            break;
        case ZP_B_TCP: case ZP_B_UDP: case ZP_B_ICMPV4: case ZP_B_ICMPV6: {
            const bool v4 = prev == BS_V4 || prev == BS_V4E;            // &[u8; 4] states
            ext = o.kind == ZP_B_TCP ? 20u : 8u;                        // as chain_extent()
            if (n < hl) {
                e = o.kind == ZP_B_TCP ? ZP_BERR_TCP_DATA : o.kind == ZP_B_UDP ? ZP_BERR_UDP_DATA
                  : o.kind == ZP_B_ICMPV4 ? ZP_BERR_ICMPV4_DATA : ZP_BERR_ICMPV6_DATA;
                break;
            }
            uint32_t start;
            if (o.kind == ZP_B_TCP) {                                    // builder.rs:438-485
                if (sl < 20) { e = ZP_BERR_TCP_SLICE; break; }
                w16(v, hl, o.h[0]); w16(v, hl + 2, o.h[1]);
                w32(v, hl + 4, o.w[0]); w32(v, hl + 8, o.w[1]);
                w8(v, hl + 12, (uint8_t)(o.b[0] << 4) | (s[12] & 0x0F));
                w8(v, hl + 12, (s[12] & 0xF0) | (o.b[1] & 0x0F));
                w8(v, hl + 13, o.b[2]);
                w16(v, hl + 14, o.h[2]);
                w16(v, hl + 18, o.h[3]);
                start = (uint32_t)(s[12] >> 4) * 4;
            } else if (o.kind == ZP_B_UDP) {                             // builder.rs:492-527
                if (sl < 8) { e = ZP_BERR_UDP_SLICE; break; }
                w16(v, hl, o.h[0]); w16(v, hl + 2, o.h[1]); w16(v, hl + 4, o.h[2]);
                start = 8;
            } else {                                                     // builder.rs:534-604
                if (sl < 8) { e = ZP_BERR_ICMP_SLICE; break; }
                w8(v, hl, o.b[0]); w8(v, hl + 1, o.b[1]);
                start = 8;
            }
            if (has) {                                                   // set_payload
                if (start > sl) { e = ZP_BERR_PANIC; break; }            // tcp.rs:109-114
                if (sl - start < dl) {
                    e = o.kind == ZP_B_ICMPV4 ? ZP_BERR_ICMPV4_PAYLOAD
                      : o.kind == ZP_B_ICMPV6 ? ZP_BERR_ICMPV6_PAYLOAD : ZP_BERR_TCP_PAYLOAD;
                    break;
                }
                ext = start + dl > ext ? start + dl : ext;
                bcopy<MODE>(v, hl + start, d, dl, lane, true);
            }
            const uint32_t proto = o.kind == ZP_B_TCP ? 6u : o.kind == ZP_B_UDP ? 17u : 58u;
            const uint32_t acc = o.kind == ZP_B_ICMPV4 ? 0u : pseudo(o, v4, proto, sl);
            const uint32_t at = o.kind == ZP_B_TCP ? 16u : o.kind == ZP_B_UDP ? 6u : 2u;
            w8(v, hl + at, 0); w8(v, hl + at + 1, 0);                    // set_checksum
            uint16_t c;
            if constexpr (MODE == ZB_M_COOP) {
                wave_sync();
                c = bcsum_lds(stage, shift, hl, n, acc, lane);
            } else if constexpr (MODE == ZB_M_GLOBAL) {
                c = bcsum_seq((const uint8_t*)v.b, hl, n, acc);
            } else {
                c = wc.csum(hl, acc);
            }
            w16(v, hl + at, c);
            hl += o.kind == ZP_B_TCP ? start : 8u;
            break;
        }
        default:
            e = ZP_BERR_TRANSITION;
        }
        const uint32_t top = base + ext < n ? base + ext : n;
        hw = top > hw ? top : hw;
        if (e) { *hl_out = hl; *done_out = k; *hw_out = hw; return e; }
    }
    *hl_out = hl;
    *done_out = nops;
    *hw_out = hw;
    return 0;
}

#define ZB_KATTR __launch_bounds__(64 * ZB_WAVES) __attribute__((amdgpu_waves_per_eu(ZB_WPE)))
#define ZB_SCAN 16             // 64-frame spans scanned per wave of the pending pass

// Frame i on a group of ZB_G lanes (slot = the group's LDS slot).
__device__ __forceinline__ void build_frame(uint64_t i, int slot, int lane,
                                            uint8_t* __restrict__ arena,
                                            const uint64_t* __restrict__ offs,
                                            const uint32_t* __restrict__ lens,
                                            const zp_build_op* __restrict__ ops,
                                            const uint32_t* __restrict__ op_start,
                                            const uint8_t* __restrict__ data,
                                            zp_build_result* __restrict__ results,
                                            uint8_t (*lds_all)[ZB_LDS],
                                            zp_build_op (*lds_ops)[ZB_OPS]) {
    const uint32_t len = lens[i];
    uint8_t* const g = arena + offs[i];
    const uint32_t o0 = op_start[i], o1 = op_start[i + 1];
    const uint32_t shift = (uint32_t)((uintptr_t)g & 15);
    const bool coop = len + shift <= ZB_LDS;
    uint8_t ZB_LDSP* lds = (uint8_t ZB_LDSP*)lds_all[slot];
    uint8_t* const a0 = (uint8_t*)((uintptr_t)g & ~(uintptr_t)15);
    const uint32_t nch = (len + shift + 15) >> 4;
    uint32_t hl = 0, done = 0, hw = 0;
    int err = ZP_BERR_TRANSITION;
    const uint32_t nops = o1 >= o0 ? o1 - o0 : 0u;
    OpSrc src{(const zp_build_op ZB_LDSP*)lds_ops[slot], ops + o0};
    {
        // one round trip: the chain's first ops (4 lanes per 64-B op) and,
        // in LDS mode, the 16-B chunks holding the frame (bytes of
        // neighbours in the edge chunks are staged but never written back)
        const uint32_t nq = 4 * (nops < ZB_OPS ? nops : ZB_OPS);
        for (uint32_t q = lane; q < nq; q += ZB_G)
            ((zb_u32x4 ZB_LDSP*)lds_ops[slot])[q] = ((const zb_u32x4*)(ops + o0))[q];
        if (coop)
            for (uint32_t c = lane; c < nch; c += ZB_G)
                *(zb_u32x4 ZB_LDSP*)(lds + 16 * c) = *(const zb_u32x4*)(a0 + 16 * c);
        wave_sync();
    }
    if (coop) {
        BView<uint8_t ZB_LDSP*> v{lds + shift, len, true};
        if (o1 >= o0)
            err = run_chain<ZB_M_COOP>(v, lds, shift, src, nops, NoWin{}, data, lane, &hl, &done,
                                       &hw);
        if (hw) {
            wave_sync();
            // write back frame bytes [0, hw): whole chunks as 16-B stores, the
            // partial edge chunks byte by byte (never a neighbour's byte)
            const uint32_t end = shift + hw;          // in staged coordinates
            for (uint32_t c = lane; c < (end + 15) >> 4; c += ZB_G) {
                const uint32_t lo = 16 * c, hi = lo + 16;
                if (lo >= shift && hi <= end) {
                    *(zb_u32x4*)(a0 + lo) = *(const zb_u32x4 ZB_LDSP*)(lds + lo);
                } else {
                    for (uint32_t q = lo < shift ? shift : lo; q < (hi < end ? hi : end); ++q)
                        a0[q] = lds[q];
                }
            }
        }
    } else {
        BView<uint8_t*> v{g, len, true};
        if (o1 >= o0)
            err = run_chain<ZB_M_GLOBAL>(v, lds, shift, src, nops, NoWin{}, data, lane, &hl, &done,
                                         &hw);
    }
    if (results && lane == 0) {
        zp_build_result r;
        r.header_len = hl;
        r.err = (uint8_t)err;
        r.ops_done = (uint8_t)(done > 255 ? 255 : done);
        r.reserved = 0;
        results[i] = r;
    }
}

// The pending pass: the frames the lane path left marked ZB_PENDING. Each
// wave scans ZB_SCAN spans of 64 results (one ballot per span) and builds the
// pending ones ZB_F at a time, a lane group per frame; the groups of a wave
// run side by side (same instructions for same-shaped chains). A small grid:
// with nothing pending the pass is one read of the results.
__global__ void ZB_KATTR
zp_build_kernel(uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, uint64_t n, const zp_build_op* __restrict__ ops,
                const uint32_t* __restrict__ op_start, const uint8_t* __restrict__ data,
                zp_build_result* __restrict__ results) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_all[ZB_WAVES * ZB_F][ZB_LDS];
    __shared__ __attribute__((aligned(16))) zp_build_op lds_ops[ZB_WAVES * ZB_F][ZB_OPS];
    const int w = threadIdx.x >> 6, l64 = threadIdx.x & 63;
    const int g = l64 / ZB_G, lane = l64 & (ZB_G - 1);
    const int slot = w * ZB_F + g;
    for (uint32_t k = 0; k < ZB_SCAN; ++k) {
        const uint64_t base = (((uint64_t)blockIdx.x * ZB_WAVES + w) * ZB_SCAN + k) * 64;
        if (base >= n) break;                                      // wave-uniform
        const uint64_t idx = base + l64;
        uint64_t m = __ballot(idx < n && results[idx].err == ZB_PENDING);
        while (m) {                                                // wave-uniform
            // group q takes the q-th lowest pending frame of the span
            int bit = -1;
#pragma unroll
            for (int q = 0; q < ZB_F; ++q) {
                const int b = m ? __builtin_ctzll(m) : -1;
                if (q == g) bit = b;
                m &= m - 1;                                        // m == 0 stays 0
            }
            if (bit >= 0)
                build_frame(base + (uint64_t)bit, slot, lane, arena, offs, lens, ops, op_start,
                            data, results, lds_all, lds_ops);
            wave_sync();                                           // slot reused next round
        }
    }
}


// ---------------------------------------------------------------------------
// Lane-per-frame path (zp_build_fast_kernel). A wave takes 64 consecutive
// frames through the packed stream of the parse kernel (zp_stream.h): every
// byte read once by full 1 KiB loads, each frame's word sum V of its 16-B
// chunks, its first ZP_WIN bytes (the window) and last chunk in LDS. Each
// lane then runs its own chain on its window (ZB_M_WIN) when every byte the
// chain can touch lies in the window; the L4 checksum comes from the stream
// sum corrected by the window chunks the chain changed, so the payload is
// never read a second time. Frames the window cannot hold (long headers,
// payload copies past it, frames under 64 B or over 64 KiB) are marked
// ZB_PENDING and built by the lane-group kernel in a second launch.
// ---------------------------------------------------------------------------

// A lane's chain in global memory (address space 1: the compiler knows these
// loads cannot alias the LDS stores of the chain and may issue them early).
struct OpGlobal {
    const zp_build_op* g;
    __device__ __forceinline__ zp_build_op get(uint32_t k) const {
        const ZP_GLOBAL zp_u32x4* q = (const ZP_GLOBAL zp_u32x4*)(g + k);
        const zp_u32x4 t[4] = {q[0], q[1], q[2], q[3]};
        zp_build_op o;
        __builtin_memcpy(&o, t, sizeof o);
        return o;
    }
    __device__ __forceinline__ uint32_t kind(uint32_t k) const {
        return *(const ZP_GLOBAL uint8_t*)(g + k);
    }
    // what chain_extent needs of op k: bytes 0-3 (kind, b[0], b[1]) and data_len
    __device__ __forceinline__ uint2 head(uint32_t k) const {
        const ZP_GLOBAL uint32_t* q = (const ZP_GLOBAL uint32_t*)(g + k);
        return make_uint2(q[0], q[7]);
    }
};

// ZB_OP_PREFETCH: the heads of a chain's first ZB_OPH ops are loaded before
// the stream (their latency hides behind it), chain_extent reads them from
// registers after it; later ops are loaded then.
#define ZB_OPH 4
struct OpHeads {
    OpGlobal og;
    uint2 h[ZB_OPH];
    __device__ __forceinline__ void load(uint32_t nops) {
#pragma unroll
        for (uint32_t k = 0; k < ZB_OPH; ++k) h[k] = k < nops ? og.head(k) : make_uint2(0, 0);
    }
    __device__ __forceinline__ uint2 head(uint32_t k) const {
        uint2 r = make_uint2(0, 0);
#pragma unroll
        for (uint32_t j = 0; j < ZB_OPH; ++j) if (k == j) r = h[j];
        return k < ZB_OPH ? r : og.head(k);
    }
    // run_chain's accessors: kinds from the heads, whole ops from HBM
    __device__ __forceinline__ zp_build_op get(uint32_t k) const { return og.get(k); }
    __device__ __forceinline__ uint32_t kind(uint32_t k) const {
        return k < ZB_OPH ? (head(k).x & 0xFFu) : og.kind(k);
    }
};

__device__ __forceinline__ uint32_t sad4(uint4 q) {
    return sad16(q.w, sad16(q.z, sad16(q.y, sad16(q.x, 0u))));
}

// After the stream each lane copies its window out of the swizzled
// [chunk][rank] cells into a private contiguous region of the same LDS
// (ZB_RSTRIDE = ZP_WIN / 4 + 1 dwords per lane, an odd count: the lanes'
// accesses to a same offset fall in 64 different banks), so the chain
// addresses bytes directly.
#define ZB_RSTRIDE (ZP_WIN + 4)
static_assert(64 * ZB_RSTRIDE <= (ZP_WIN_CH + 1) * 64 * 16, "regions must fit the window LDS");

__device__ __forceinline__ uint4 ld_region(const uint8_t ZB_LDSP* r, uint32_t at) {
    const uint32_t ZB_LDSP* d = (const uint32_t ZB_LDSP*)(r + at);
    return make_uint4(d[0], d[1], d[2], d[3]);
}

// internet_checksum(bytes[l4 .. len], acc) (checksum.rs:5-29) from the
// stream: V of the frame's chunks with the window chunks' changes applied,
// minus the chunks before l4 and the bytes past the frame end. With V the
// word sum at even ARENA addresses, the reference's word sum W satisfies
// W = V (segment starts at an odd address) or W == 256 V (mod 65535); the
// fold of S = acc + W depends only on S mod 65535 and on S == 0 (exact for
// frames up to 64 KiB, the only ones this path takes).
// The folded checksum from V (arena parity, exact), the accumulator and the
// parity of the segment's first byte.
__device__ __forceinline__ uint16_t fold_v(uint32_t V, uint32_t acc, bool even) {
    if (acc == 0 && V == 0) return 0xFFFF;                 // S == 0: !fold(0)
    uint32_t w = V % 65535u;
    if (even) w = (w * 256u) % 65535u;
    const uint32_t r = (acc % 65535u + w) % 65535u;
    return (uint16_t)~(r ? r : 65535u);
}

struct WinCsum {
    const uint8_t ZB_LDSP* region;    // the lane's window, from A & ~15
    uint4 tail;                       // the frame's last chunk (original bytes)
    uintptr_t ga;
    uint32_t shift, len, nchw, fsum;
    bool wo;                          // window-only stream (ZB_SKIP_PAY): no bytes past the end
    uint32_t vorig[ZP_WIN_CH];
    // what csum() saw, for a payload copied past the window after the chain
    // (coop_payload): the checksum is then refolded with the copy's V change
    mutable uint32_t cs_V, cs_acc, cs_l4;
    __device__ uint16_t csum(uint32_t l4, uint32_t acc) const {
        const uint32_t y4 = l4 + shift, c4 = y4 >> 4;
        uint32_t vall = fsum, before = 0;
#pragma unroll
        for (uint32_t c = 0; c < ZP_WIN_CH; ++c) {
            if (c < nchw) {
                const uint4 q = ld_region(region, 16 * c);
                const uint32_t vn = sad4(q);
                vall += vn - vorig[c];
                if (c < c4) before += vn;
                else if (c == c4) before += range_sum(q, 0, y4 & 15);
            }
        }
        const uint32_t he = wo ? 0u : (len + shift) & 15u;
        const uint32_t ex = he ? range_sum(tail, he, 16u) : 0u;
        const uint32_t V = vall - before - ex;
        cs_V = V; cs_acc = acc; cs_l4 = l4;
        return fold_v(V, acc, !((ga + l4) & 1));
    }
};

// Upper bound of the bytes a chain can read or write (from its ops alone;
// the offsets the writers derive from the buffer are the values the chain
// itself wrote: ihl, data offset, extension lengths).
template <class Ops>
__device__ __forceinline__ uint32_t chain_extent(const Ops& ops, uint32_t nops, uint32_t* pay_at = nullptr,
                             uint32_t* pay_len = nullptr, bool* pay_ovl = nullptr) {
    // With pay_at: the final L4 op's payload copy is left out of the extent
    // and reported as [*pay_at, *pay_at + *pay_len) (frame offsets).
    uint32_t hl = 0, top = 0;
    if (pay_at) { *pay_at = 0; *pay_len = 0; }
    if (pay_ovl) *pay_ovl = false;
    for (uint32_t k = 0; k < nops; ++k) {
        const uint2 hd = ops.head(k);
        struct { uint32_t kind; uint8_t b[2]; uint32_t data_len; } o;
        o.kind = hd.x & 0xFFu;
        o.b[0] = (uint8_t)(hd.x >> 8);
        o.b[1] = (uint8_t)(hd.x >> 16);
        o.data_len = hd.y;
        const uint32_t dl = o.data_len != ZP_BUILD_NO_DATA ? o.data_len : 0u;
        uint32_t ext = 0, adv = 0;
        switch (o.kind) {
        case ZP_B_ETHERNET: case ZP_B_ETHERNET_VLAN: case ZP_B_ETHERNET_QINQ:
            ext = 22; hl = 0;
            adv = o.kind == ZP_B_ETHERNET ? 14 : o.kind == ZP_B_ETHERNET_VLAN ? 18 : 22;
            break;
        case ZP_B_ARP: ext = 28; adv = 28; break;
        case ZP_B_IPV4: adv = (o.b[1] & 15u) * 4; ext = adv > 20 ? adv : 20; break;
        case ZP_B_IPV6: ext = 40; adv = 40; break;
        case ZP_B_HOP_BY_HOP: case ZP_B_DEST_OPTS1: case ZP_B_DEST_OPTS2:
            ext = 2 + dl; adv = ((uint32_t)o.b[1] + 1) * 8; break;
        case ZP_B_ROUTING: ext = 8 + dl; adv = ((uint32_t)o.b[1] + 1) * 8; break;
        case ZP_B_FRAGMENT: ext = 8; adv = 8; break;
        case ZP_B_AUTH: ext = 12 + dl; adv = ((uint32_t)o.b[1] + 2) * 4; break;
        case ZP_B_TCP: {
            const uint32_t st = (o.b[0] & 15u) * 4;
            ext = st + dl > 20 ? st + dl : 20; adv = st;
            if (pay_at && k + 1 == nops && dl) {
                *pay_at = hl + st; *pay_len = dl; ext = st > 20 ? st : 20;
                if (pay_ovl) *pay_ovl = st < 20;         // (the payload overwrites header fields)
            }
            break;
        }
        default:                                         // UDP, ICMPv4, ICMPv6
            ext = 8 + dl; adv = 8;
            if (pay_at && k + 1 == nops && dl) { *pay_at = hl + 8; *pay_len = dl; ext = 8; }
            break;
        }
        top = hl + ext > top ? hl + ext : top;
        hl += adv;
        if (hl > 0x100000u) return ~0u;                  // no window holds that
    }
    return top;
}

#define ZB_FAST_WPE 3          // at least 3 waves per SIMD (168 VGPRs): the LDS allows 3

// Wave-cooperative segments: lane j owns cnt_j chunks; the wave walks the
// concatenation of all lanes' chunks in items of 64 (lane l of item i takes
// virtual chunk 64 i + l, its owner j found by a binary search over the
// owners' exclusive prefix with ds_bpermute), ZB_COOP_U items at a time:
// load(j, k, live) issues chunk k of owner j's loads for all of them first,
// then use(data, j, k, live) consumes them (stores, a u32 contribution), so
// ZB_COOP_U items' loads are in flight per wave. Returns, per lane, the
// wrapping sum of its own chunks' contributions (running-sum differences:
// no segmented reduction). Every lane must be active (DPP scans, bpermute).
#define ZB_COOP_U 8            // round 4, with ZB_SKIP_PAY and ZB_COPY_X4: 8 vs 4 P = 1000 -1.1 %, P = 200 -0.2 %; round 3, without ZB_PIPE_SEARCH 1: 2.04 / 3.52 ms, 2: 1.95 / 3.16, 4: 1.99 / 3.26, 8: 2.11 / 3.52 (P = 200 / 1000); with it 2: 1.85 / 2.80, 4: 1.82 / 2.71, 8: 1.82 / 2.70
// ZB_PIPE_SEARCH: the owner search of the next ZB_COOP_U items (dependent
// ds_bpermute round trips) is issued while this round's loads are in flight,
// not after its stores.
template <class D, class L, class U>
__device__ __forceinline__ uint32_t wave_segments(uint32_t cnt, int lane, L&& load, U&& use) {
    const uint32_t incl = wave_scan(cnt), pre = incl - cnt;
    const uint32_t T = rdl(incl, 63);
    uint32_t carry = 0, p_pre = 0, p_end = 0;
    auto search = [&](uint32_t base, uint32_t* jj, uint32_t* kk) {
#pragma unroll
        for (int u = 0; u < ZB_COOP_U; ++u) {
            const uint32_t g = base + 64u * u + (uint32_t)lane;
            uint32_t j = 0;                              // largest j with pre_j <= g
#pragma unroll
            for (uint32_t st = 32; st; st >>= 1)
                j = bperm(pre, j + st) <= g ? j + st : j;
            jj[u] = j;
            kk[u] = g - bperm(pre, j);
        }
    };
    uint32_t jj[ZB_COOP_U], kk[ZB_COOP_U];
    if (T) search(0, jj, kk);
    for (uint32_t base = 0; base < T; base += 64 * ZB_COOP_U) {
        D d[ZB_COOP_U];
#pragma unroll
        for (int u = 0; u < ZB_COOP_U; ++u)
            d[u] = load(jj[u], kk[u], base + 64u * u + (uint32_t)lane < T);
        uint32_t ju[ZB_COOP_U], ku[ZB_COOP_U];
#pragma unroll
        for (int u = 0; u < ZB_COOP_U; ++u) ju[u] = jj[u], ku[u] = kk[u];
        if (base + 64 * ZB_COOP_U < T) search(base + 64 * ZB_COOP_U, jj, kk);
#pragma unroll
        for (int u = 0; u < ZB_COOP_U; ++u) {
            const uint32_t b = base + 64u * u;
            const uint32_t v = use(d[u], ju[u], ku[u], b + (uint32_t)lane < T);
            const uint32_t inc = wave_scan(v), exc = inc - v;
            const uint32_t xp = bperm(exc, (pre - b) & 63u), xe = bperm(exc, (incl - b) & 63u);
            if (pre >= b && pre < b + 64) p_pre = carry + xp;
            if (incl >= b && incl < b + 64) p_end = carry + xe;
            carry += rdl(inc, 63);
        }
    }
    if (pre >= T) p_pre = carry;
    if (incl >= T) p_end = carry;
    return p_end - p_pre;
}

__device__ __forceinline__ uint64_t bperm64(uint64_t v, uint32_t r) {
    return ((uint64_t)bperm((uint32_t)(v >> 32), r) << 32) | bperm((uint32_t)v, r);
}

// Bytes [s, e) of the 16-B chunk q to the 16-B-aligned address X (0 <= s <
// e <= 16) in at most one byte, one short, one 1-4 dword and one short + byte
// store per lane, instead of one byte store per byte: a wave whose lanes end
// their ranges anywhere in a chunk issues a handful of store instructions, not
// up to 15 (ZB_WIDE_EDGES).
__device__ __forceinline__ uint32_t q_dw(uint4 q, uint32_t i) {
    return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w;
}
__device__ __forceinline__ void store_bytes(uintptr_t X, uint4 q, uint32_t s, uint32_t e) {
    uint32_t b = s;
    if ((b & 1u) && b < e) {
        *(ZP_GLOBAL uint8_t*)(X + b) = (uint8_t)(q_dw(q, b >> 2) >> (8 * (b & 3u)));
        ++b;
    }
    if ((b & 2u) && b + 2 <= e) {
        *(ZP_GLOBAL uint16_t*)(X + b) = (uint16_t)(q_dw(q, b >> 2) >> 16);
        b += 2;
    }
    const uint32_t nd = (b & 3u) == 0 && b < e ? (e - b) >> 2 : 0u;
    if (nd) {
        const uint32_t i = b >> 2;
        const uint32_t d0 = q_dw(q, i), d1 = q_dw(q, i + 1), d2 = q_dw(q, i + 2);
        if (nd == 1) *(ZP_GLOBAL uint32_t*)(X + b) = d0;
        else if (nd == 2) *(ZP_GLOBAL zp_u32x2*)(X + b) = zp_u32x2{d0, d1};
        else if (nd == 3) {
            typedef unsigned u32x3 __attribute__((ext_vector_type(3)));
            *(ZP_GLOBAL u32x3*)(X + b) = u32x3{d0, d1, d2};
        } else {
            *(ZP_GLOBAL zp_u32x4*)(X + b) = zp_u32x4{q.x, q.y, q.z, q.w};
        }
        b += 4 * nd;
    }
    if (b + 2 <= e) {                                  // b is 4-aligned here
        *(ZP_GLOBAL uint16_t*)(X + b) = (uint16_t)q_dw(q, b >> 2);
        b += 2;
    }
    if (b < e) *(ZP_GLOBAL uint8_t*)(X + b) = (uint8_t)(q_dw(q, b >> 2) >> (8 * (b & 3u)));
}

// f packs the chunk's byte range [lo, m) (bits 0-4, 5-9), the source's
// offset in its dword (10-11) and nb (12): 8 chunks in flight per lane
struct CopyChunk { uint32_t x[5]; uintptr_t X; uint32_t f; };
struct SumChunk { uint4 q; uint32_t l, h, neg; };

// The payload bytes past the header, for every lane whose chain ends in a
// payload copy that reaches past its window (go): destination [D0, D1) of
// its frame from the blob at src (the payload's first byte). The whole wave
// moves 16-B chunks of [D0 & ~15, D1): coalesced loads of the blob, full
// 16-B stores, partial ones by store_bytes. With ZB_PAY_HDR the copy starts
// at the payload start D0 (the chain copies nothing) and the first chunk,
// when D0 is not 16-B aligned, is left to the caller (it also holds header
// bytes, among them the checksum refolded after this pass); without it D0 is
// the window end W (16-B aligned) and the chain copies the window part.
// Returns the copy's change of the frame's V (arena parity) past the window:
// V of the copied bytes at their destination minus V of the bytes they
// replace in [W, D1). The latter is summed over the shorter of two ranges of
// original bytes, read before any copy is written (a first pass): [W, D1)
// itself (kind A), or the frame's bytes after the copy [D1, FE) (kind B),
// then V(W, D1) = the frame's stream sum - its window chunks - V(D1, FE) -
// the bytes past its end in its last chunk (cB, from the kept original
// chunk: in HBM they are the next frame's, whose lane may be rewriting
// them). Window-only (wo) frames take kind B with cB = 0.
__device__ __forceinline__ uint32_t coop_payload(bool go, uintptr_t W, uintptr_t D0, uintptr_t D1,
                                                 uintptr_t FE, uintptr_t src, uint32_t cB,
                                                 int lane, bool wo, bool defer0,
                                                 bool known = false, uint32_t vrep = 0) {
    const uint32_t mw = go ? (uint32_t)(D1 - W) : 0u;    // copied bytes past the window
    const bool kA = !wo && mw <= (uint32_t)(FE - D1);   // wo frames: kind B (W..D1 never read)
    const uintptr_t R0 = kA ? W : (D1 & ~(uintptr_t)15);
    // (known: V(W, D1) is vrep, from the stream; a copy to the frame end
    // reads nothing either)
    const bool rd = go && !known && (kA || FE > D1);
    const uint32_t rlo = rd ? (uint32_t)((kA ? W : D1) - R0) : 0u;
    const uint32_t rhi = rd ? (uint32_t)((kA ? D1 : FE) - R0) : 0u;
    // pass 1: original bytes (loads only)
    const uint32_t vo = wave_segments<SumChunk>(
        (rhi + 15) >> 4, lane,
        [&](uint32_t j, uint32_t k, bool live) {
            const uintptr_t r0 = bperm64(R0, j);
            SumChunk c;
            const uint32_t lo = bperm(rlo, j), hi = bperm(rhi, j);
            c.neg = bperm(kA ? 1u : 0u, j);
            const uint32_t a = 16u * k;
            c.l = lo > a ? lo - a : 0u;
            c.h = hi - a < 16u ? hi - a : 16u;
            c.q = live ? ldg16(r0 + a) : make_uint4(0, 0, 0, 0);
            return c;
        },
        [&](const SumChunk& c, uint32_t, uint32_t, bool live) {
            if (!live) return 0u;
            const uint32_t v = range_sum(c.q, c.l, c.h);
            return c.neg ? 0u - v : v;
        });
    // pass 2: the copy, chunks of [D0a, D1); chunk k holds bytes [lo, m)
    const uintptr_t D0a = D0 & ~(uintptr_t)15;
    const uint32_t o0 = go ? (uint32_t)(D0 - D0a) : 0u;
    const uint32_t mc = go ? (uint32_t)(D1 - D0) : 0u;
    const uint32_t vn = wave_segments<CopyChunk>(
        (o0 + mc + 15) >> 4, lane,
        [&](uint32_t j, uint32_t k, bool live) {
            const uintptr_t d0 = bperm64(D0a, j), s0 = bperm64(src, j);
            const uint32_t oj = bperm(o0, j), m_all = oj + bperm(mc, j);
            CopyChunk c;
            const uint32_t lo = k == 0 ? oj : 0u;
            const uint32_t m = m_all - 16u * k < 16u ? m_all - 16u * k : 16u;
            // source of the chunk's byte 0 (for a first chunk with header
            // bytes, before src: only dwords holding copied bytes are loaded)
            const uintptr_t S = s0 + 16u * k - oj, sb = S & ~(uintptr_t)3;
            const uintptr_t slo = S + lo, send = S + m;
            const uint32_t sh = (uint32_t)(S & 3);
            c.X = d0 + 16u * k;
            // Whole chunks: one dwordx4 from the dword below S; the 5th dword
            // is the next lane's first when it holds this copy's next chunk
            // (nb), else its own dword load. Partial chunks: dword loads
            // inside the copied range (no read outside the blob range).
            const bool full = lo == 0 && m == 16;
            const uint32_t jn = bperm(j, (uint32_t)lane + 1u), kn = bperm(k, (uint32_t)lane + 1u);
            const bool ln = bperm(live ? 1u : 0u, (uint32_t)lane + 1u) != 0u;
            const bool nb = lane < 63 && ln && jn == j && kn == k + 1u;
            c.f = lo | m << 5 | sh << 10 | (nb ? 1u << 12 : 0u);
            if (live && full) {
                const zp_u32x4 v = *(const ZP_GLOBAL zp_u32x4*)sb;
                c.x[0] = v.x; c.x[1] = v.y; c.x[2] = v.z; c.x[3] = v.w;
                c.x[4] = sh && !nb ? *(const ZP_GLOBAL uint32_t*)(sb + 16u) : 0u;
            } else {
#pragma unroll
                for (int u = 0; u < 5; ++u) {
                    const uintptr_t a = sb + 4u * u;
                    c.x[u] = live && a < send && a + 4u > slo ? *(const ZP_GLOBAL uint32_t*)a : 0u;
                }
            }
            return c;
        },
        [&](const CopyChunk& c, uint32_t, uint32_t, bool live) {
            const uint32_t x1 = bperm(c.x[0], (uint32_t)lane + 1u);   // every lane (bpermute)
            const uint32_t lo = c.f & 31u, m = (c.f >> 5) & 31u, sh = (c.f >> 10) & 3u;
            const bool full = lo == 0 && m == 16;
            const uint32_t x4 = full && (c.f >> 12 & 1u) ? x1 : c.x[4];
            if (!live) return 0u;
            const uint4 q = make_uint4(__builtin_amdgcn_alignbyte(c.x[1], c.x[0], sh),
                                       __builtin_amdgcn_alignbyte(c.x[2], c.x[1], sh),
                                       __builtin_amdgcn_alignbyte(c.x[3], c.x[2], sh),
                                       __builtin_amdgcn_alignbyte(x4, c.x[3], sh));
            if (full) {
                *(ZP_GLOBAL zp_u32x4*)c.X = zp_u32x4{q.x, q.y, q.z, q.w};
            } else if (!(defer0 && lo)) {         // (a first chunk with header bytes: the caller)
                store_bytes(c.X, q, lo, m);
            }
            return range_sum(q, lo, m);
        });
    return vn + (known ? 0u - vrep : go && !kA ? cB + vo : vo);
}

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ZB_FAST_WPE)))
zp_build_fast_kernel(uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                     const uint32_t* __restrict__ lens, uint64_t n,
                     const zp_build_op* __restrict__ ops, const uint32_t* __restrict__ op_start,
                     const uint8_t* __restrict__ data, zp_build_result* __restrict__ results) {
    __shared__ WaveLds lds;
    // the 3 chunks before each frame's last one (the previous frame's bytes
    // in a frame's first 64-B sector)
    __shared__ uint4 t4[64 * ZP_T4N];
    __shared__ uint32_t cmid[64];                      // running sum at each frame's mark
    constexpr bool T4 = true;
    const int lane = threadIdx.x & 63;
    const uint64_t t = blockIdx.x;
    if (t * 64 >= n) return;
    const uintptr_t fallback = (uintptr_t)&zp_safe_chunk;
    uint4* win = &lds.win[0];
    uint4* tail = &lds.win[ZP_WIN_CH * 64];
    uint32_t len;
    uintptr_t ga;
    // The chain's bounds before the stream: their latency hides behind it
    // (-1 to -2 %; the ops themselves in registers spill: +5 %).
    const uint64_t ip = t * 64 + lane, ipc = ip < n ? ip : n - 1;
    const uint32_t pf0 = op_start[ipc], pf1 = op_start[ipc + 1];
    load_desc(arena, offs, lens, n, t, lane, len, ga);
    TileState s;
    OpHeads oh{OpGlobal{ops + (ip < n ? pf0 : 0u)}};
    oh.load(ip < n && pf1 >= pf0 ? pf1 - pf0 : 0u);
    // A frame whose final payload copy replaces at least as many bytes past
    // the window as follow the copy streams its window only (wo): the bytes
    // the copy replaces are never read, the ones after it are read by the
    // copy's first pass, and the L4 sum is built from the new window, the
    // copy and those. Deciding it needs the chain's heads before the stream.
    // The other payload frames mark the copy's end in the stream (ZB_MARK):
    // the running sum there gives V of the bytes the copy replaces, so the
    // copy needs no first pass over them.
    bool wo = false;
    uint32_t mark = ~0u;
    if (ip < n && pf1 >= pf0 && len >= 64 && len <= ZP_GIANT) {
        uint32_t pa = 0, pl = 0;
        const uint32_t sh0 = (uint32_t)(ga & 15);
        const uint32_t wl0 = len < ZP_WIN - sh0 ? len : ZP_WIN - sh0;
        if (chain_extent(oh, pf1 - pf0, &pa, &pl) <= wl0 && pl && pa + pl > wl0) {
            const uint32_t pe = pa + pl;
            wo = pe <= len && pe - wl0 >= len - pe;
            if (!wo && pe < len) mark = pe;
        }
    }
    tile_setup(s, t, len, ga, n, lane, lds, wo, mark);
    uint4 va[ZP_G];
    uint32_t ka[ZP_G];
    issue_group<ZP_G, T4>(0, s.nitems, s.cur, s.R, lane, fallback, va, ka);
    consume_group<ZP_G, T4>(0, s.nitems, lane, va, ka, win, tail, lds.cend, s.run, t4, cmid);
    for (uint32_t i0 = ZP_G; i0 < s.nitems; i0 += ZP_G) {
        issue_group<ZP_G, T4>(i0, s.nitems, s.cur, s.R, lane, fallback, va, ka);
        consume_group<ZP_G, T4>(i0, s.nitems, lane, va, ka, win, tail, lds.cend, s.run, t4, cmid);
    }
    wave_lds_fence();                                  // windows written by other lanes
    // Every lane stays to the neighbour exchange after the chains; frames
    // that are not built here are marked pending for the lane-group pass.
    const uint64_t i = t * 64 + lane;
    uint32_t o0 = 0, nops = 0;
    bool fast = false;
    bool pay = false;                                  // payload bytes past the window
    uint32_t pay_at = 0, pay_len = 0;
    bool pay_ovl = false;                              // a TCP payload over its own header
    if (s.live) {
        o0 = pf0;
        const uint32_t o1 = pf1;
        nops = o1 >= o0 ? o1 - o0 : 0u;
        // A final payload copy may reach past the window: the headers must
        // fit it; the copy's bytes past it go straight to HBM after the chain.
        if (o1 >= o0 && len >= 64 && !s.giant) {
            fast = chain_extent(oh, nops, &pay_at, &pay_len, &pay_ovl) <= s.wlen;
            pay = fast && pay_len && pay_at + pay_len > s.wlen;
        }
        if (!fast) {
            zp_build_result r;
            r.header_len = 0; r.err = (uint8_t)ZB_PENDING; r.ops_done = 0; r.reserved = 0;
            results[i] = r;
        }
    }
    // ph: the wave copy moves the whole payload (ZB_PAY_HDR), unless it
    // overwrites the L4 header's own fields (a TCP data offset below 5: the
    // chain keeps the reference's write order then)
    const bool ph = pay && !pay_ovl;
    const uint32_t rank = s.rank & 63u;
    const uint32_t nch = (len + s.shift + 15) >> 4;
    WinCsum wc;
    uint4 cells[ZP_WIN_CH];
    uint4 ptail = make_uint4(0, 0, 0, 0);              // the previous frame's last chunk
    if (fast) {
        wc.ga = s.ga;
        wc.shift = s.shift;
        wc.len = len;
        wc.nchw = nch < ZP_WIN_CH ? nch : ZP_WIN_CH;
        wc.fsum = lds.cend[s.rank] - (s.rank ? lds.cend[s.rank - 1] : 0u);
        wc.tail = tail[rank];
        wc.wo = wo;
        ptail = tail[(rank - 1) & 63u];
#pragma unroll
        for (uint32_t c = 0; c < ZP_WIN_CH; ++c) {
            cells[c] = c < wc.nchw ? win[c * 64 + ((rank ^ c) & 63u)] : make_uint4(0, 0, 0, 0);
            wc.vorig[c] = sad4(cells[c]);
        }
    }
    wave_lds_fence();                                  // every lane holds its cells
    uint8_t ZB_LDSP* region = (uint8_t ZB_LDSP*)win + lane * ZB_RSTRIDE;
    uint32_t hl = 0, done = 0, hw = 0, doff = 0, lkind = 0;
    int err = 0;
    if (fast) {
#pragma unroll
        for (uint32_t c = 0; c < ZP_WIN_CH; ++c) {
            uint32_t ZB_LDSP* d = (uint32_t ZB_LDSP*)(region + 16 * c);
            d[0] = cells[c].x; d[1] = cells[c].y; d[2] = cells[c].z; d[3] = cells[c].w;
        }
        wc.region = region;
        BView<uint8_t ZB_LDSP*> v{region + s.shift, len, true};
        // The whole wave copies the payload after the chain (coop_payload;
        // without ZB_PAY_HDR the chain writes its window part), and the L4
        // checksum is refolded with that copy's V change below.
        if (pay) v.lim = ph ? pay_at : s.wlen;
        err = run_chain<ZB_M_WIN>(v, (const uint8_t ZB_LDSP*)nullptr, s.shift, oh, nops, wc,
                                  data, lane, &hl, &done, &hw, &doff, &lkind);
    }
    {
        // A copy that does not fit the frame failed in the chain before any
        // byte was written (err != 0): nothing to copy then. The headers fit
        // the window and the payload reaches past it.
        const bool go = pay && err == 0;
        const uint32_t pe = pay_at + pay_len;
        const uint32_t c0 = (s.shift + pay_at) >> 4;   // window chunk of the payload's start
        uintptr_t src = 0;
        uint32_t cB = 0, vw = 0, Vw = 0;
        if (go) {
            src = (uintptr_t)data + doff + (ph ? 0u : s.wlen - pay_at);   // (the chain's last op)
#pragma unroll
            for (uint32_t c = 0; c < ZP_WIN_CH; ++c) {
                Vw += wc.vorig[c];
                // ph: V of the window's bytes from the payload start on, as
                // the checksum saw them (original bytes, or header bytes an
                // invalid chain wrote there); the copy's sum has the new ones
                if (ph && c >= c0)
                    vw += range_sum(ld_region(region, 16 * c), c == c0 ? (s.shift + pay_at) & 15u : 0u, 16u);
            }
            const uint32_t he = wo ? 0u : (len + s.shift) & 15u;
            cB = Vw + (he ? range_sum(wc.tail, he, 16u) : 0u) - wc.fsum;   // 0 for wo frames
        }
        // a marked frame: V of the original bytes [W, D1) from the running
        // sum at the copy's end minus the frame's start and window chunks
        const bool known = go && mark != ~0u;
        const uint32_t vrep = known ? cmid[rank] - (rank ? lds.cend[rank - 1] : 0u) - Vw : 0u;
        const uint32_t delta = coop_payload(go, s.ga + s.wlen, s.ga + (ph ? pay_at : s.wlen),
                                            s.ga + pe, s.ga + len, src, cB, lane, wo, true,
                                            known, vrep);
        if (go) {                                      // refold the L4 checksum
            const uint32_t k4 = lkind;                  // the chain's last op (go: all ran)
            const uint32_t at = k4 == ZP_B_TCP ? 16u : k4 == ZP_B_UDP ? 6u : 2u;
            const uint16_t c = fold_v(wc.cs_V + delta - vw, wc.cs_acc, !((s.ga + wc.cs_l4) & 1));
            region[s.shift + wc.cs_l4 + at] = (uint8_t)(c >> 8);
            region[s.shift + wc.cs_l4 + at + 1] = (uint8_t)c;
            // The chunk holding the payload's first byte, when it also holds
            // header bytes: those from the region (the checksum refolded),
            // the payload's from the blob again (a line the copy has just
            // read), one whole-chunk store.
            const uint32_t o0 = (s.shift + pay_at) & 15u;
            if (ph && o0) {
                const uint4 h = ld_region(region, 16 * c0);
                const uintptr_t S = src - o0, sb = S & ~(uintptr_t)3;
                const uint32_t sh2 = (uint32_t)(S & 3);
                uint32_t x[5];
#pragma unroll
                for (int u = 0; u < 5; ++u) {
                    const uintptr_t a = sb + 4u * u;
                    x[u] = a < S + 16u && a + 4u > src ? *(const ZP_GLOBAL uint32_t*)a : 0u;
                }
                const uint32_t p[4] = {__builtin_amdgcn_alignbyte(x[1], x[0], sh2),
                                       __builtin_amdgcn_alignbyte(x[2], x[1], sh2),
                                       __builtin_amdgcn_alignbyte(x[3], x[2], sh2),
                                       __builtin_amdgcn_alignbyte(x[4], x[3], sh2)};
                const uint32_t hh[4] = {h.x, h.y, h.z, h.w};
                uint32_t m[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t keep = byte_mask(4 * i, 0, (int)o0);      // header bytes
                    m[i] = (hh[i] & keep) | (p[i] & ~keep);
                }
                *(ZP_GLOBAL zp_u32x4*)((s.ga & ~(uintptr_t)15) + 16u * c0) = zp_u32x4{m[0], m[1], m[2], m[3]};
            }
        }
    }
    // Write-back of frame bytes [0, hw) from the region: whole 16-B chunks as
    // one store, edge chunks byte by byte (never a byte another lane writes).
    // A store that covers part of a 64-B HBM sector costs ~2.4 x a whole one
    // (read-modify-write), so the lane completes its header's
    // sectors where it can: the last one to its end with the frame's
    // unchanged bytes from the window, and the first one from its start with
    // the previous frame's unchanged tail (the 3 chunks before its last one,
    // kept by the stream, and the shared chunk from the window) when that
    // frame ends exactly here and its lane writes nothing there.
    const uintptr_t a0 = s.ga & ~(uintptr_t)15;
    const uint32_t sh = s.shift;
    const bool pay_go = pay && err == 0;               // the chain copied the payload
    const uint32_t hwc = hw < s.wlen ? hw : s.wlen;               // hw <= extent <= wlen
    uint32_t end = fast ? sh + hwc : sh;                          // window coordinates
    if (fast) {
        const uint32_t se = (uint32_t)(((s.ga + hwc + 63) & ~(uintptr_t)63) - a0);
        const uint32_t fe = sh + len;
        const uint32_t e1 = se < fe ? se : fe;                    // never past the frame
        if (hwc && e1 <= sh + s.wlen) end = e1;                   // bytes in the window
    }
    // the payload's chunks (from the one holding its first byte) are the copy's
    if (pay_go && ph) {
        const uint32_t pc = (sh + pay_at) & ~15u;
        end = end < pc ? end : pc;
    }
    // the previous lane's frame and where its writes end (all lanes active)
    const uintptr_t wend = pay_go ? s.ga + pay_at + pay_len : a0 + end;
    const uint32_t pl = lane ? (uint32_t)lane - 1u : 0u;
    const uintptr_t pA = ((uintptr_t)bperm((uint32_t)(s.ga >> 32), pl) << 32) |
                         bperm((uint32_t)s.ga, pl);
    const uintptr_t pW = ((uintptr_t)bperm((uint32_t)(wend >> 32), pl) << 32) |
                         bperm((uint32_t)wend, pl);
    const uint32_t pLen = bperm(s.live ? len : 0u, pl);
    const uintptr_t S0 = s.ga & ~(uintptr_t)63;
    // (a window-only previous frame has no last chunks in t4 / tail)
    const bool pwo = bperm(wo ? 1u : 0u, pl) != 0u;
    const bool pre = fast && lane && hwc && (s.ga & 63u) && pLen >= 64 && pLen <= ZP_GIANT && !pwo &&
                     pA + pLen == s.ga &&
                     ((((s.ga - 1) & ~(uintptr_t)15) - S0) >> 4) <= (uintptr_t)ZP_T4N &&
                     S0 >= pA && S0 >= pW;
    // One loop over the lane's chunks from S0 (pre) or a0, in address order:
    // the previous frame's kept chunks, then the region's. As two loops (the
    // kept chunks first) the first sector reached HBM twice for ~40 % of the
    // frames (TCC_EA0_WRREQ 9.14M for 7.09M sectors per 4M c3 frames; one
    // loop 7.41M, 1.045 x, and -2 % time: profiles/r06_build_writes_unified.log).
    const uint32_t npre = pre ? (uint32_t)((a0 - S0) >> 4) : 0u;
    const uintptr_t lastc = (s.ga - 1) & ~(uintptr_t)15;          // the previous frame's last chunk
    const uint32_t ntot = npre + ((end + 15) >> 4);
    for (uint32_t k = 0; k < ntot; ++k) {
        if (k < npre) {
            const uintptr_t X = S0 + 16u * k;
            const uint32_t d = (uint32_t)((lastc - X) >> 4);      // 0..3
            const uint4 q = d == 0 ? ptail : t4[(rank - 1) * ZP_T4N + d - 1];
            *(ZP_GLOBAL zp_u32x4*)X = zp_u32x4{q.x, q.y, q.z, q.w};
            continue;
        }
        const uint32_t c = k - npre;
        const uint32_t lo = 16 * c, hi = lo + 16;
        if ((lo >= sh || (pre && c == 0)) && hi <= end) {
            const uint4 q = ld_region(region, lo);
            *(ZP_GLOBAL zp_u32x4*)(a0 + lo) = zp_u32x4{q.x, q.y, q.z, q.w};
        } else {
            const uint32_t bs = lo < sh ? sh : lo, be = hi < end ? hi : end;
            if (bs < be) store_bytes(a0 + lo, ld_region(region, lo), bs - lo, be - lo);
        }
    }
    if (!fast) return;
    zp_build_result r;
    r.header_len = hl;
    r.err = (uint8_t)err;
    r.ops_done = (uint8_t)(done > 255 ? 255 : done);
    r.reserved = 0;
    results[i] = r;
}

extern "C" int zp_build_batch_device(uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                     uint64_t n, const zp_build_op* ops, const uint32_t* op_start,
                                     const uint8_t* data, zp_build_result* results,
                                     void* stream) {
    if (n == 0) return 0;
    if (!arena || !offs || !lens || !ops || !op_start) {
        snprintf(zp__errbuf(), 256, "zp_build_batch_device: null pointer");
        return -1;
    }
    const uint64_t per_block = (uint64_t)ZB_WAVES * ZB_SCAN * 64;   // pending pass
    const uint64_t blocks = (n + per_block - 1) / per_block;
    const uint64_t fast_blocks = (n + 63) / 64;
    if (blocks > 0x7FFFFFFFull || fast_blocks > 0x7FFFFFFFull) {
        snprintf(zp__errbuf(), 256, "zp_build_batch_device: batch too large");
        return -1;
    }
    hipStream_t st = (hipStream_t)stream;
    // The lane-per-frame pass needs a per-frame "pending" mark: the results
    // array, or a stream-ordered scratch copy when the caller passes none.
    zp_build_result* res = results;
    if (!res && hipMallocAsync((void**)&res, n * sizeof(zp_build_result), st) != hipSuccess) {
        snprintf(zp__errbuf(), 256, "zp_build_batch_device: scratch allocation failed");
        return -2;
    }
    hipLaunchKernelGGL(zp_build_fast_kernel, dim3((unsigned)fast_blocks), dim3(64), 0, st, arena,
                       offs, lens, n, ops, op_start, data, res);
    hipLaunchKernelGGL(zp_build_kernel, dim3((unsigned)blocks), dim3(64 * ZB_WAVES), 0, st, arena,
                       offs, lens, n, ops, op_start, data, res);
    if (!results) (void)hipFreeAsync(res, st);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(zp__errbuf(), 256, "zp_build_kernel launch: %s", hipGetErrorString(e));
        return -2;
    }
    return 0;
}
