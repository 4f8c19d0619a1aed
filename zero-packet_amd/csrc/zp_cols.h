// zp_cols.h — the column views of one parsed frame (include/zero_packet.h,
// zp_col), shared by the stand-alone column kernel (zp_fields.hip) and the
// fused parse + columns kernel (zp_parse.hip). Each getter cites the
// reference line it follows; `rd(x)` returns frame byte x from wherever the
// caller staged it.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/zero_packet.h"

typedef unsigned zp_u32x2 __attribute__((ext_vector_type(2)));

struct ColPtrs {
    uint8_t* p[ZP_COL_COUNT];
};

// The parse result of one frame with every field unpacked: the kernels'
// working form, packed into the 8-B zp_record (include/zero_packet.h) only
// at the store. final_nh / inner_final_nh are IPv6Reader::final_next_header
// (ipv6.rs:219-227) of the outer / ip_in_ip IPv6.
struct zp_rec_full {
    uint32_t flags;
    uint8_t err, eth_len, final_nh, inner_final_nh;
    uint32_t inner_off, l4_off;
    uint32_t chain;      // the outer chain's inline code (offs bits 18-31), 0: none
};

// The outer chain goes inline (ZP_CHAIN_INLINE, include/zero_packet.h): the
// walk found it short and in RFC order, there is no ip_in_ip header and an
// L4 reader gives final_next_header.
__device__ __forceinline__ bool zp_chain_inline(const zp_rec_full& r) {
    return (r.flags & (ZP_F_EXT | ZP_F_IP_IN_IP)) == ZP_F_EXT &&
           (r.flags & (ZP_F_TCP | ZP_F_UDP | ZP_F_ICMPV4 | ZP_F_ICMPV6)) &&
           (r.chain & (ZP_CHAIN_INLINE >> 18)) && r.l4_off <= ZP_L4_NEAR_MAX;
}

// The 8-B record (include/zero_packet.h); an L4 reader past ZP_L4_NEAR_MAX
// takes the far-L4 form: Ethernet code 3, the whole offset in `offs`.
__device__ __forceinline__ zp_u32x2 zp_pack(const zp_rec_full& r) {
    if (r.err) return zp_u32x2{(uint32_t)r.err << 26, 0u};
    const bool far = r.l4_off > ZP_L4_NEAR_MAX;
    const uint32_t code = far ? ZP_ETH_CODE_FAR : (uint32_t)(r.eth_len - 14) >> 2;
    const uint32_t hi = zp_chain_inline(r) ? r.chain : r.inner_off;
    return zp_u32x2{r.flags | code << 24, far ? r.l4_off : r.l4_off | (hi << 18)};
}

// A reader R gives frame byte x as rd(x), and bytes [x, x + 4) as one
// little-endian dword rd.le4(x) when rd.has4(x) (all four staged: two dword
// reads and a v_alignbyte instead of four byte reads).

// n bytes [x, x + n) packed little-endian (n <= 4): memory order preserved.
template <class R>
__device__ __forceinline__ uint32_t rd_le(R& rd, uint32_t x, int n) {
    if (rd.has4(x)) {
        const uint32_t v = rd.le4(x);
        return n >= 4 ? v : v & ((1u << (8 * n)) - 1u);
    }
    uint32_t v = 0;
    for (int k = 0; k < n; ++k) v |= rd(x + k) << (8 * k);
    return v;
}
// Big-endian fields.
template <class R>
__device__ __forceinline__ uint32_t rd16(R& rd, uint32_t x) {
    const uint32_t v = rd_le(rd, x, 2);
    return ((v & 0xFFu) << 8) | (v >> 8);
}
template <class R>
__device__ __forceinline__ uint32_t rd32(R& rd, uint32_t x) {
    return __builtin_bswap32(rd_le(rd, x, 4));
}

template <typename T>
__device__ __forceinline__ void st(const ColPtrs& c, int col, uint64_t i, T v) {
    if (c.p[col]) ((T*)c.p[col])[i] = v;
}

// 16-byte address entry: IPv4 (4 bytes + zeros) or IPv6 (16 bytes).
template <class R>
__device__ __forceinline__ void col_addr(const ColPtrs& c, int col, uint64_t i, R& rd, uint32_t x,
                                         bool v6) {
    if (!c.p[col]) return;
    uint4 v;
    v.x = rd_le(rd, x, 4);
    v.y = v6 ? rd_le(rd, x + 4, 4) : 0u;
    v.z = v6 ? rd_le(rd, x + 8, 4) : 0u;
    v.w = v6 ? rd_le(rd, x + 12, 4) : 0u;
    ((uint4*)c.p[col])[i] = v;
}

template <class R>
__device__ __forceinline__ void col_mac(const ColPtrs& c, int col, uint64_t i, R& rd, uint32_t x) {
    if (!c.p[col]) return;
    uint16_t* d = (uint16_t*)(c.p[col] + 6 * i);
    d[0] = (uint16_t)rd_le(rd, x, 2);
    d[1] = (uint16_t)rd_le(rd, x + 2, 2);
    d[2] = (uint16_t)rd_le(rd, x + 4, 2);
}

// Writes entry i of every requested column for one frame: record r (ok =
// parsed without error, with an Ethernet reader), frame length len.
template <class R>
__device__ __forceinline__ void emit_columns(R& rd, const zp_rec_full& r, bool ok, uint32_t len,
                                             uint64_t i, const ColPtrs& c) {
    // Absent readers / errors read 0.
    uint8_t ipv = 0, proto = 0, ttl = 0, tos = 0, iv = 0, iproto = 0, l4p = 0, tflags = 0;
    uint8_t ity = 0, icode = 0;
    uint16_t ety = 0, tci = 0, tci2 = 0, oper = 0, iplen = 0, sport = 0, dport = 0, win16 = 0;
    uint16_t l4ck = 0;
    uint32_t ipid = 0, seq = 0, ack = 0, poff = 0;
    const uint4 z = make_uint4(0, 0, 0, 0);
    if (ok) {
        const uint32_t hl = r.eth_len;
        col_mac(c, ZP_COL_DEST_MAC, i, rd, 0);                          // ethernet.rs:195-198
        col_mac(c, ZP_COL_SRC_MAC, i, rd, 6);                           // ethernet.rs:201-204
        ety = (uint16_t)rd16(rd, hl - 2);                              // ethernet.rs:209-212
        const uint32_t tp = rd16(rd, 12);
        if (tp == 0x8100) tci = (uint16_t)rd16(rd, 14);                // ethernet.rs:218-229
        else if (tp == 0x88A8) {                                      // ethernet.rs:232-244
            tci = (uint16_t)rd16(rd, 14);
            tci2 = (uint16_t)rd16(rd, 18);
        }
        if (r.flags & ZP_F_ARP) oper = (uint16_t)rd16(rd, hl + 6);     // arp.rs:174-177
        if (r.flags & (ZP_F_IPV4 | ZP_F_IPV6)) {
            const bool v6 = (r.flags & ZP_F_IPV6) != 0;
            ipv = (uint8_t)(rd(hl) >> 4);                          // ipv4.rs:148 / ipv6.rs:173
            col_addr(c, ZP_COL_SRC_ADDR, i, rd, hl + (v6 ? 8 : 12), v6);
            col_addr(c, ZP_COL_DEST_ADDR, i, rd, hl + (v6 ? 24 : 16), v6);
            if (!v6) {
                proto = (uint8_t)rd(hl + 9);                       // ipv4.rs:204-207
                ttl = (uint8_t)rd(hl + 8);                         // ipv4.rs:198-201
                tos = (uint8_t)rd(hl + 1);                         // ipv4.rs:160-169
                ipid = rd16(rd, hl + 4);                               // ipv4.rs:180-183
                iplen = (uint16_t)rd16(rd, hl + 2);                    // ipv4.rs:174-177
            } else {
                proto = r.final_nh;                                   // ipv6.rs:219-227
                ttl = (uint8_t)rd(hl + 7);                         // ipv6.rs:237-240
                const uint32_t b0 = rd(hl), b1 = rd(hl + 1);
                tos = (uint8_t)(((b0 & 0x0F) << 4) | (b1 >> 4));      // ipv6.rs:181-186
                ipid = ((b1 & 0x0F) << 16) | rd16(rd, hl + 2);         // ipv6.rs:189-196
                iplen = (uint16_t)rd16(rd, hl + 4);                    // ipv6.rs:199-202
            }
        } else {
            if (c.p[ZP_COL_SRC_ADDR]) ((uint4*)c.p[ZP_COL_SRC_ADDR])[i] = z;
            if (c.p[ZP_COL_DEST_ADDR]) ((uint4*)c.p[ZP_COL_DEST_ADDR])[i] = z;
        }
        if (r.flags & ZP_F_IP_IN_IP) {
            const bool v6 = (r.flags & ZP_F_IP_IN_IP_V6) != 0;
            const uint32_t p = r.inner_off;
            iv = (uint8_t)(rd(p) >> 4);
            col_addr(c, ZP_COL_INNER_SRC_ADDR, i, rd, p + (v6 ? 8 : 12), v6);
            col_addr(c, ZP_COL_INNER_DEST_ADDR, i, rd, p + (v6 ? 24 : 16), v6);
            iproto = v6 ? r.inner_final_nh : (uint8_t)rd(p + 9);
        } else {
            if (c.p[ZP_COL_INNER_SRC_ADDR]) ((uint4*)c.p[ZP_COL_INNER_SRC_ADDR])[i] = z;
            if (c.p[ZP_COL_INNER_DEST_ADDR]) ((uint4*)c.p[ZP_COL_INNER_DEST_ADDR])[i] = z;
        }
        const uint32_t l4f = r.flags & (ZP_F_TCP | ZP_F_UDP | ZP_F_ICMPV4 | ZP_F_ICMPV6);
        if (l4f) {
            const uint32_t p = r.l4_off;
            uint32_t hlen = 8;
            if (l4f == ZP_F_TCP) {
                l4p = 6;
                sport = (uint16_t)rd16(rd, p);                         // tcp.rs:151-154
                dport = (uint16_t)rd16(rd, p + 2);                     // tcp.rs:157-160
                seq = rd32(rd, p + 4);                                 // tcp.rs:163-170
                ack = rd32(rd, p + 8);                                 // tcp.rs:172-179
                const uint32_t b12 = rd16(rd, p + 12);
                tflags = (uint8_t)(b12 & 0xFF);                       // tcp.rs:193-196
                hlen = (b12 >> 12) * 4;                               // tcp.rs:217-220
                win16 = (uint16_t)rd16(rd, p + 14);                    // tcp.rs:199-202
                l4ck = (uint16_t)rd16(rd, p + 16);                     // tcp.rs:205-208
            } else if (l4f == ZP_F_UDP) {
                l4p = 17;
                sport = (uint16_t)rd16(rd, p);                         // udp.rs:113-116
                dport = (uint16_t)rd16(rd, p + 2);                     // udp.rs:119-122
                l4ck = (uint16_t)rd16(rd, p + 6);                      // udp.rs:125-128
            } else {
                l4p = l4f == ZP_F_ICMPV4 ? 1 : 58;
                const uint32_t tc = rd16(rd, p);
                ity = (uint8_t)(tc >> 8);                             // icmpv4.rs:102-105
                icode = (uint8_t)(tc & 0xFF);                         // icmpv4.rs:108-111
                l4ck = (uint16_t)rd16(rd, p + 2);                      // icmpv4.rs:114-117
            }
            if (hlen <= len - p) poff = p + hlen;                     // tcp.rs:235-243
        }
    } else {
        if (c.p[ZP_COL_DEST_MAC]) {
            uint16_t* d = (uint16_t*)(c.p[ZP_COL_DEST_MAC] + 6 * i);
            d[0] = 0; d[1] = 0; d[2] = 0;
        }
        if (c.p[ZP_COL_SRC_MAC]) {
            uint16_t* d = (uint16_t*)(c.p[ZP_COL_SRC_MAC] + 6 * i);
            d[0] = 0; d[1] = 0; d[2] = 0;
        }
        if (c.p[ZP_COL_SRC_ADDR]) ((uint4*)c.p[ZP_COL_SRC_ADDR])[i] = z;
        if (c.p[ZP_COL_DEST_ADDR]) ((uint4*)c.p[ZP_COL_DEST_ADDR])[i] = z;
        if (c.p[ZP_COL_INNER_SRC_ADDR]) ((uint4*)c.p[ZP_COL_INNER_SRC_ADDR])[i] = z;
        if (c.p[ZP_COL_INNER_DEST_ADDR]) ((uint4*)c.p[ZP_COL_INNER_DEST_ADDR])[i] = z;
    }
    st<uint16_t>(c, ZP_COL_ETHERTYPE, i, ety);
    st<uint16_t>(c, ZP_COL_VLAN_TCI, i, tci);
    st<uint16_t>(c, ZP_COL_VLAN_INNER_TCI, i, tci2);
    st<uint16_t>(c, ZP_COL_ARP_OPER, i, oper);
    st<uint8_t>(c, ZP_COL_IP_VERSION, i, ipv);
    st<uint8_t>(c, ZP_COL_PROTOCOL, i, proto);
    st<uint8_t>(c, ZP_COL_TTL, i, ttl);
    st<uint8_t>(c, ZP_COL_TOS, i, tos);
    st<uint32_t>(c, ZP_COL_IP_ID, i, ipid);
    st<uint16_t>(c, ZP_COL_IP_LEN, i, iplen);
    st<uint8_t>(c, ZP_COL_INNER_VERSION, i, iv);
    st<uint8_t>(c, ZP_COL_INNER_PROTOCOL, i, iproto);
    st<uint8_t>(c, ZP_COL_L4_PROTO, i, l4p);
    st<uint16_t>(c, ZP_COL_SRC_PORT, i, sport);
    st<uint16_t>(c, ZP_COL_DEST_PORT, i, dport);
    st<uint32_t>(c, ZP_COL_TCP_SEQ, i, seq);
    st<uint32_t>(c, ZP_COL_TCP_ACK, i, ack);
    st<uint8_t>(c, ZP_COL_TCP_FLAGS, i, tflags);
    st<uint16_t>(c, ZP_COL_TCP_WINDOW, i, win16);
    st<uint8_t>(c, ZP_COL_ICMP_TYPE, i, ity);
    st<uint8_t>(c, ZP_COL_ICMP_CODE, i, icode);
    st<uint16_t>(c, ZP_COL_L4_CHECKSUM, i, l4ck);
    st<uint32_t>(c, ZP_COL_PAYLOAD_OFF, i, poff);
}
