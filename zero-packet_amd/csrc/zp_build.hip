// zp_build.hip — batched PacketBuilder.
//
// Reference: builder.rs:55-909 (the typestate chain) and the writers it
// calls: EthernetWriter ethernet.rs:19-129, ArpWriter arp.rs:7-119,
// IPv4Writer ipv4.rs:8-127, IPv6Writer ipv6.rs:8-133, Options/Routing/
// Fragment/AuthenticationHeaderWriter (extensions/*.rs), TcpWriter
// tcp.rs:7-130, UdpWriter udp.rs:7-92, Icmpv4Writer icmpv4.rs:10-81,
// Icmpv6Writer icmpv6.rs:7-78; checksums checksum.rs:5-69.
//
// One wave per frame (a chain is a serial program, but its payload copy and
// the L4 checksum over the rest of the buffer are wave-wide work). Frames up
// to ZB_CAP bytes (+ alignment) are staged in LDS: the wave loads the frame,
// executes the chain on the LDS copy and writes back only the bytes the chain
// can have changed. Longer frames run in place in global memory, every lane
// executing the same chain on the same bytes.
//
// The chain's scalar steps run on every lane with identical values (every
// lane stores the same byte to the same address), so each lane reads back
// its own writes and no cross-lane ordering is needed except after the
// cooperative steps (staging, copies), which end with a wave barrier.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/zero_packet.h"

extern "C" char* zp__errbuf(void);

#define ZB_WAVES 4
#define ZB_CAP 2048            // frame bytes staged in LDS per wave
#define ZB_LDS (ZB_CAP + 32)   // + the frame's offset in its first 16-B chunk

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

// Frame view for the chain: a generic pointer to the staged (LDS) or the
// in-place (global) bytes. Every lane executes every access.
struct BView {
    uint8_t* b;
    uint32_t n;
    uint32_t hw;      // one past the highest byte written (LDS write-back bound)
};

__device__ __forceinline__ void w8(BView& v, uint32_t i, uint32_t x) {
    v.b[i] = (uint8_t)x;
    v.hw = i + 1 > v.hw ? i + 1 : v.hw;
}
__device__ __forceinline__ void w16(BView& v, uint32_t i, uint32_t x) {
    w8(v, i, x >> 8);
    w8(v, i + 1, x);
}
__device__ __forceinline__ void w32(BView& v, uint32_t i, uint32_t x) {
    w16(v, i, x >> 16);
    w16(v, i + 2, x);
}
__device__ __forceinline__ void wbytes(BView& v, uint32_t i, const uint8_t* s, int k) {
    for (int q = 0; q < k; ++q) w8(v, i + q, s[q]);
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Copies `len` bytes of the data blob to frame offset `at`: lane-strided in
// LDS mode (then a wave barrier), every lane all bytes in global mode.
__device__ void bcopy(BView& v, uint32_t at, const uint8_t* src, uint32_t len, bool coop,
                      int lane) {
    if (coop) {
        for (uint32_t q = lane; q < len; q += 64) v.b[at + q] = src[q];
        wave_sync();
    } else {
        for (uint32_t q = 0; q < len; ++q) v.b[at + q] = src[q];
    }
    if (len) v.hw = at + len > v.hw ? at + len : v.hw;
}

// internet_checksum(bytes[s0 .. n], acc) (checksum.rs:5-29, u32 wrap): the
// u32 sum is associative, so a lane-strided partial sum + wave reduction is
// bit-identical to the reference's sequential loop.
__device__ uint16_t bcsum(const BView& v, uint32_t s0, uint32_t acc, bool coop, int lane) {
    const uint32_t len = v.n - s0;
    const uint32_t words = len >> 1;
    uint32_t sum = 0;
    const uint32_t first = coop ? (uint32_t)lane : 0u, step = coop ? 64u : 1u;
    for (uint32_t w = first; w < words; w += step)
        sum += ((uint32_t)v.b[s0 + 2 * w] << 8) | v.b[s0 + 2 * w + 1];
    if (coop) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) sum += (uint32_t)__shfl_xor((int)sum, off);
    }
    sum += acc;
    if (len & 1) sum += (uint32_t)v.b[v.n - 1] << 8;
    while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
    return (uint16_t)~sum;
}

// checksum.rs:43-69 over 4- or 16-byte addresses.
__device__ __forceinline__ uint32_t pseudo(const zp_build_op& o, int alen, uint32_t proto,
                                           uint32_t length) {
    uint32_t s = 0;
    for (int k = 0; k < alen; k += 2) s += ((uint32_t)o.src[k] << 8) | o.src[k + 1];
    for (int k = 0; k < alen; k += 2) s += ((uint32_t)o.dst[k] << 8) | o.dst[k + 1];
    return s + proto + length;
}

// Executes one chain (all checks of the reference, in its order). Returns
// the zp_build_err; *hl_out = header_len after the last Ok op.
__device__ int run_chain(BView& v, const zp_build_op* __restrict__ ops, uint32_t nops,
                         const uint8_t* __restrict__ data, bool coop, int lane, uint32_t* hl_out,
                         uint32_t* done_out) {
    int st = BS_RAW;
    for (uint32_t k = 0; k < nops; ++k) {            // typestate (compile time in Rust)
        st = bnext(st, ops[k].kind);
        if (st < 0) { *hl_out = 0; *done_out = 0; return ZP_BERR_TRANSITION; }
    }
    st = BS_RAW;
    uint32_t hl = 0;
    const uint32_t n = v.n;
    for (uint32_t k = 0; k < nops; ++k) {
        const zp_build_op o = ops[k];
        const int prev = st;
        st = bnext(st, o.kind);
        const bool has = o.data_len != ZP_BUILD_NO_DATA;
        const uint32_t dl = has ? o.data_len : 0u;
        const uint8_t* d = data + o.data_off;
        const uint32_t sl = n - hl;                  // &mut bytes[header_len..]
        uint8_t* s = v.b + hl;
        int e = 0;
        switch (o.kind) {
        case ZP_B_ETHERNET: case ZP_B_ETHERNET_VLAN: case ZP_B_ETHERNET_QINQ: {
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
            if (n < hl) { e = ZP_BERR_ARP_DATA; break; }
            if (sl < 28) { e = ZP_BERR_ARP_SLICE; break; }
            w16(v, hl, o.h[0]); w16(v, hl + 2, o.h[1]); w8(v, hl + 4, o.b[0]); w8(v, hl + 5, o.b[1]);
            w16(v, hl + 6, o.h[2]);
            wbytes(v, hl + 8, o.src, 6); wbytes(v, hl + 14, o.src + 6, 4);
            wbytes(v, hl + 18, o.dst, 6); wbytes(v, hl + 24, o.dst + 6, 4);
            hl += 28;
            break;
        case ZP_B_IPV4: {                                                // builder.rs:248-292
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
            if (n < hl) { e = o.kind == ZP_B_HOP_BY_HOP ? ZP_BERR_HBH_DATA : ZP_BERR_DEST_DATA; break; }
            if (sl < 8) { e = ZP_BERR_OPTIONS_SLICE; break; }
            w8(v, hl, o.b[0]);
            w8(v, hl + 1, o.b[1]);
            if (dl < 6) { e = ZP_BERR_OPTIONS_MIN; break; }             // options.rs:53-68
            if ((uint32_t)s[1] * 8 != dl) { e = ZP_BERR_OPTIONS_MATCH; break; }
            if (2 + dl > sl) { e = ZP_BERR_OPTIONS_EXCEED; break; }
            bcopy(v, hl + 2, d, dl, coop, lane);
            hl += ((uint32_t)s[1] + 1) * 8;
            break;
        case ZP_B_ROUTING:                                               // builder.rs:675-704
            if (n < hl) { e = ZP_BERR_ROUTING_DATA; break; }
            if (sl < 8) { e = ZP_BERR_ROUTING_SLICE; break; }
            w8(v, hl, o.b[0]); w8(v, hl + 1, o.b[1]); w8(v, hl + 2, o.b[2]); w8(v, hl + 3, o.b[3]);
            if (dl < 4) { e = ZP_BERR_ROUTING_MIN; break; }             // routing.rs:75-94
            if ((uint32_t)s[1] * 8 != dl) { e = ZP_BERR_ROUTING_MATCH; break; }
            if (8 + dl > sl) { e = ZP_BERR_ROUTING_EXCEED; break; }
            bcopy(v, hl + 8, d, dl, coop, lane);
            hl += ((uint32_t)s[1] + 1) * 8;
            break;
        case ZP_B_FRAGMENT: {                                            // builder.rs:711-740
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
            if (n < hl) { e = ZP_BERR_AUTH_DATA; break; }
            if (sl < 12) { e = ZP_BERR_AUTH_SLICE; break; }
            w8(v, hl, o.b[0]); w8(v, hl + 1, o.b[1]); w8(v, hl + 2, 0); w8(v, hl + 3, 0);
            w32(v, hl + 4, o.w[0]);
            w32(v, hl + 8, o.w[1]);
            if (12 + dl > sl) { e = ZP_BERR_AUTH_EXCEED; break; }       // authentication.rs:84-92
            bcopy(v, hl + 12, d, dl, coop, lane);
            hl += ((uint32_t)s[1] + 2) * 4;
            break;
        case ZP_B_TCP: case ZP_B_UDP: case ZP_B_ICMPV4: case ZP_B_ICMPV6: {
            const bool v4 = prev == BS_V4 || prev == BS_V4E;            // &[u8; 4] states
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
                bcopy(v, hl + start, d, dl, coop, lane);
            }
            const uint32_t proto = o.kind == ZP_B_TCP ? 6u : o.kind == ZP_B_UDP ? 17u : 58u;
            const uint32_t acc = o.kind == ZP_B_ICMPV4 ? 0u : pseudo(o, v4 ? 4 : 16, proto, sl);
            const uint32_t at = o.kind == ZP_B_TCP ? 16u : o.kind == ZP_B_UDP ? 6u : 2u;
            w8(v, hl + at, 0); w8(v, hl + at + 1, 0);                    // set_checksum
            if (coop) wave_sync();
            const uint16_t c = bcsum(v, hl, acc, coop, lane);
            w16(v, hl + at, c);
            hl += o.kind == ZP_B_TCP ? start : 8u;
            break;
        }
        default:
            e = ZP_BERR_TRANSITION;
        }
        if (e) { *hl_out = hl; *done_out = k; return e; }
    }
    *hl_out = hl;
    *done_out = nops;
    return 0;
}

__global__ void __launch_bounds__(64 * ZB_WAVES)
zp_build_kernel(uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, uint64_t n, const zp_build_op* __restrict__ ops,
                const uint32_t* __restrict__ op_start, const uint8_t* __restrict__ data,
                zp_build_result* __restrict__ results) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_all[ZB_WAVES][ZB_LDS];
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    // wave-uniform frame index (scalar loads of its descriptors and ops)
    const uint64_t i = (uint64_t)blockIdx.x * ZB_WAVES +
                       (uint32_t)__builtin_amdgcn_readfirstlane(wid);
    if (i >= n) return;
    const uint32_t len = lens[i];
    uint8_t* const g = arena + offs[i];
    const uint32_t o0 = op_start[i], o1 = op_start[i + 1];
    const uint32_t shift = (uint32_t)((uintptr_t)g & 15);
    const bool coop = len + shift <= ZB_LDS;
    uint8_t* lds = lds_all[wid];
    BView v;
    v.n = len;
    v.hw = 0;
    uint8_t* const a0 = (uint8_t*)((uintptr_t)g & ~(uintptr_t)15);
    const uint32_t nch = (len + shift + 15) >> 4;
    if (coop) {
        // stage the 16-B chunks holding the frame (bytes of neighbours in the
        // edge chunks are staged but never written back)
        for (uint32_t c = lane; c < nch; c += 64)
            *(uint4*)(lds + 16 * c) = *(const uint4*)(a0 + 16 * c);
        wave_sync();
        v.b = lds + shift;
    } else {
        v.b = g;
    }
    uint32_t hl = 0, done = 0;
    const int err = o1 >= o0 ? run_chain(v, ops + o0, o1 - o0, data, coop, lane, &hl, &done)
                             : ZP_BERR_TRANSITION;
    if (coop && v.hw) {
        wave_sync();
        // write back frame bytes [0, hw): whole chunks as 16-B stores, the
        // partial edge chunks byte by byte (never a neighbour's byte)
        const uint32_t end = shift + v.hw;            // in staged coordinates
        for (uint32_t c = lane; c < (end + 15) >> 4; c += 64) {
            const uint32_t lo = 16 * c, hi = lo + 16;
            if (lo >= shift && hi <= end) {
                *(uint4*)(a0 + lo) = *(const uint4*)(lds + lo);
            } else {
                for (uint32_t q = lo < shift ? shift : lo; q < (hi < end ? hi : end); ++q)
                    a0[q] = lds[q];
            }
        }
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

extern "C" int zp_build_batch_device(uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                                     uint64_t n, const zp_build_op* ops, const uint32_t* op_start,
                                     const uint8_t* data, zp_build_result* results,
                                     void* stream) {
    if (n == 0) return 0;
    if (!arena || !offs || !lens || !ops || !op_start) {
        snprintf(zp__errbuf(), 256, "zp_build_batch_device: null pointer");
        return -1;
    }
    const uint64_t blocks = (n + ZB_WAVES - 1) / ZB_WAVES;
    if (blocks > 0x7FFFFFFFull) {
        snprintf(zp__errbuf(), 256, "zp_build_batch_device: batch too large");
        return -1;
    }
    hipLaunchKernelGGL(zp_build_kernel, dim3((unsigned)blocks), dim3(64 * ZB_WAVES), 0,
                       (hipStream_t)stream, arena, offs, lens, n, ops, op_start, data, results);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(zp__errbuf(), 256, "zp_build_kernel launch: %s", hipGetErrorString(e));
        return -2;
    }
    return 0;
}
