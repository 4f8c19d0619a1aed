// zp_fields.hip — column views over parsed frames.
//
// zp_extract_columns_device gathers the reader getters of every parsed frame
// (EthernetReader ethernet.rs:195-244, ArpReader::oper arp.rs:174-177,
// IPv4Reader ipv4.rs:148-219, IPv6Reader ipv6.rs:173-256, TcpReader
// tcp.rs:151-243, UdpReader udp.rs:113-154, Icmpv4/6Reader icmpv4.rs:102-135,
// icmpv6.rs:99-132) into SoA device columns, driven by the zp_record the
// parse kernel wrote: offsets say where each reader starts, flags which
// readers exist. Column semantics: include/zero_packet.h (zp_col).
//
// One lane per frame, 256 frames per workgroup. Each lane stages the first
// 128 B of its frame (from A & ~15) in LDS with 16-B loads; headers past the
// window (deep IPv6 chains, IP-in-IP) are read from global memory. Column
// stores are one element per lane, coalesced across the wave. HBM-bound:
// per frame one or two 128-B lines in, sum of the requested column widths out.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/zero_packet.h"

extern "C" char* zp__errbuf(void);

#define FX_WIN 128                       // staged bytes per frame (from A & ~15)
#define FX_CH (FX_WIN / 16)
#define FX_BLOCK 256

static const int kColWidth[ZP_COL_COUNT] = {
    6, 6, 2, 2, 2, 2, 1, 16, 16, 1, 1, 1, 4, 2, 1, 16, 16, 1, 1, 2, 2, 4, 4, 1, 2, 1, 1, 2, 4};

extern "C" int zp_col_width(int col) {
    return col >= 0 && col < ZP_COL_COUNT ? kColWidth[col] : 0;
}

struct ColPtrs {
    uint8_t* p[ZP_COL_COUNT];
};

#define FX_GLOBAL __attribute__((address_space(1)))
typedef unsigned fx_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 fx_ld16(uintptr_t a) {
    const fx_u32x4 v = *(const FX_GLOBAL fx_u32x4*)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}

struct Hdr {
    const uint8_t* win;   // this lane's cells: byte b of chunk c at win[c * 16 * FX_BLOCK + b]
    const uint8_t* g;     // frame in global memory
    uint32_t shift, wlen;
    uint4 xc;             // past the window: one cached 16-B chunk ...
    uint32_t xi;          // ... and its index from A & ~15 (~0: none)
};

__device__ __forceinline__ uint32_t hb(Hdr& h, uint32_t x) {
    const uint32_t y = x + h.shift;
    if (x < h.wlen) return h.win[(y >> 4) * 16 * FX_BLOCK + (y & 15)];
    // Headers past the window (deep IPv6 chains, IP-in-IP): one 16-B load
    // per distinct chunk, the fields of a header share it.
    if ((y >> 4) != h.xi) {
        h.xi = y >> 4;
        h.xc = fx_ld16(((uintptr_t)h.g & ~(uintptr_t)15) + 16u * h.xi);
    }
    const uint32_t d = (y >> 2) & 3;
    const uint32_t w = d == 0 ? h.xc.x : d == 1 ? h.xc.y : d == 2 ? h.xc.z : h.xc.w;
    return (w >> (8 * (y & 3))) & 0xFFu;
}
__device__ __forceinline__ uint32_t hb16(Hdr& h, uint32_t x) {
    return (hb(h, x) << 8) | hb(h, x + 1);
}
__device__ __forceinline__ uint32_t hb32(Hdr& h, uint32_t x) {
    return (hb16(h, x) << 16) | hb16(h, x + 2);
}

template <typename T>
__device__ __forceinline__ void st(const ColPtrs& c, int col, uint64_t i, T v) {
    if (c.p[col]) ((T*)c.p[col])[i] = v;
}

// n little-endian-packed bytes [x, x + n) of the frame (n <= 4).
__device__ __forceinline__ uint32_t hbytes(Hdr& h, uint32_t x, int n) {
    uint32_t v = 0;
    for (int k = 0; k < n; ++k) v |= hb(h, x + k) << (8 * k);
    return v;
}

// 16-byte address column entry: IPv4 (4 bytes + zeros) or IPv6 (16 bytes).
__device__ __forceinline__ void st_addr(const ColPtrs& c, int col, uint64_t i, Hdr& h,
                                        uint32_t x, bool v6) {
    if (!c.p[col]) return;
    uint4 v;
    v.x = hbytes(h, x, 4);
    v.y = v6 ? hbytes(h, x + 4, 4) : 0u;
    v.z = v6 ? hbytes(h, x + 8, 4) : 0u;
    v.w = v6 ? hbytes(h, x + 12, 4) : 0u;
    ((uint4*)c.p[col])[i] = v;
}

__device__ __forceinline__ void st_mac(const ColPtrs& c, int col, uint64_t i, Hdr& h,
                                       uint32_t x) {
    if (!c.p[col]) return;
    uint16_t* d = (uint16_t*)(c.p[col] + 6 * i);
    d[0] = (uint16_t)hbytes(h, x, 2);
    d[1] = (uint16_t)hbytes(h, x + 2, 2);
    d[2] = (uint16_t)hbytes(h, x + 4, 2);
}

__global__ void __launch_bounds__(FX_BLOCK)
zp_columns_kernel(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                  const uint32_t* __restrict__ lens, const zp_record* __restrict__ recs,
                  uint64_t n, ColPtrs c) {
    __shared__ uint4 win[FX_CH * FX_BLOCK];
    const uint64_t i0 = (uint64_t)blockIdx.x * FX_BLOCK + threadIdx.x;
    // Lanes past the batch stay for the cooperative staging (no wave exits
    // early: ds_bpermute reads every lane); they load and store nothing.
    const bool live = i0 < n;
    const uint64_t i = live ? i0 : n - 1;
    const uint4* rp = (const uint4*)(recs + i);
    zp_record r;
    {
        uint4 q[2] = {rp[0], rp[1]};
        __builtin_memcpy(&r, q, sizeof r);
    }
    const bool ok = live && r.err == 0 && (r.flags & ZP_F_ETHERNET);
    const uint32_t len = ok ? lens[i] : 0u;
    const uintptr_t ga = (uintptr_t)arena + (ok ? offs[i] : 0);
    Hdr h;
    h.g = (const uint8_t*)ga;
    h.shift = (uint32_t)(ga & 15);
    // Stage only the header bytes the getters read: the last header the
    // record names ends by l4 + 20 (TCP) / inner + 40 / l3 + 40.
    uint32_t need = 22;
    if (ok) {
        const uint32_t l3 = r.eth_len + 40;
        need = l3 > need ? l3 : need;
        if (r.flags & ZP_F_IP_IN_IP) need = r.inner_off + 40 > need ? r.inner_off + 40 : need;
        if (r.flags & (ZP_F_TCP | ZP_F_UDP | ZP_F_ICMPV4 | ZP_F_ICMPV6))
            need = r.l4_off + 20 > need ? r.l4_off + 20 : need;
    }
    need = need < len ? need : len;
    h.wlen = need < FX_WIN - h.shift ? need : FX_WIN - h.shift;
    h.win = (const uint8_t*)&win[threadIdx.x];
    h.xc = make_uint4(0, 0, 0, 0);
    h.xi = ~0u;
    // Stage the chunks of [A & ~15, A + wlen) cooperatively: in item q, lane l
    // loads chunk (l & 7) of frame 8q + (l >> 3) of its wave, so one load
    // instruction reads eight whole 128-B windows instead of 64 scattered
    // 16-B pieces. Cell (chunk c, frame t) lives at win[c * FX_BLOCK + t].
    {
        const uint32_t lane = threadIdx.x & 63, wbase = threadIdx.x & ~63u;
        const uint32_t nch = len ? (h.wlen + h.shift + 15) >> 4 : 0u;
        const uintptr_t a0 = ga & ~(uintptr_t)15;
        const uint32_t a_lo = (uint32_t)a0, a_hi = (uint32_t)(a0 >> 32);
#pragma unroll
        for (uint32_t q = 0; q < 8; ++q) {
            const uint32_t f = 8 * q + (lane >> 3), ch = lane & 7;
            const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(f << 2), (int)a_lo);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(f << 2), (int)a_hi);
            const uint32_t nc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(f << 2), (int)nch);
            if (ch < nc)
                win[ch * FX_BLOCK + wbase + f] = fx_ld16((((uintptr_t)hi << 32) | lo) + 16u * ch);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }

    if (!live) return;
    // Absent readers / errors read 0.
    uint8_t ipv = 0, proto = 0, ttl = 0, tos = 0, iv = 0, iproto = 0, l4p = 0, tflags = 0;
    uint8_t ity = 0, icode = 0;
    uint16_t ety = 0, tci = 0, tci2 = 0, oper = 0, iplen = 0, sport = 0, dport = 0, win16 = 0;
    uint16_t l4ck = 0;
    uint32_t ipid = 0, seq = 0, ack = 0, poff = 0;
    const uint4 z = make_uint4(0, 0, 0, 0);
    if (ok) {
        const uint32_t hl = r.eth_len;
        st_mac(c, ZP_COL_DEST_MAC, i, h, 0);                          // ethernet.rs:195-198
        st_mac(c, ZP_COL_SRC_MAC, i, h, 6);                           // ethernet.rs:201-204
        ety = (uint16_t)hb16(h, hl - 2);                              // ethernet.rs:209-212
        const uint32_t tp = hb16(h, 12);
        if (tp == 0x8100) tci = (uint16_t)hb16(h, 14);                // ethernet.rs:218-229
        else if (tp == 0x88A8) {                                      // ethernet.rs:232-244
            tci = (uint16_t)hb16(h, 14);
            tci2 = (uint16_t)hb16(h, 18);
        }
        if (r.flags & ZP_F_ARP) oper = (uint16_t)hb16(h, hl + 6);     // arp.rs:174-177
        if (r.flags & (ZP_F_IPV4 | ZP_F_IPV6)) {
            const bool v6 = (r.flags & ZP_F_IPV6) != 0;
            ipv = (uint8_t)(hb(h, hl) >> 4);                          // ipv4.rs:148 / ipv6.rs:173
            st_addr(c, ZP_COL_SRC_ADDR, i, h, hl + (v6 ? 8 : 12), v6);
            st_addr(c, ZP_COL_DEST_ADDR, i, h, hl + (v6 ? 24 : 16), v6);
            if (!v6) {
                proto = (uint8_t)hb(h, hl + 9);                       // ipv4.rs:204-207
                ttl = (uint8_t)hb(h, hl + 8);                         // ipv4.rs:198-201
                tos = (uint8_t)hb(h, hl + 1);                         // ipv4.rs:160-169
                ipid = hb16(h, hl + 4);                               // ipv4.rs:180-183
                iplen = (uint16_t)hb16(h, hl + 2);                    // ipv4.rs:174-177
            } else {
                proto = r.final_nh;                                   // ipv6.rs:219-227
                ttl = (uint8_t)hb(h, hl + 7);                         // ipv6.rs:237-240
                const uint32_t b0 = hb(h, hl), b1 = hb(h, hl + 1);
                tos = (uint8_t)(((b0 & 0x0F) << 4) | (b1 >> 4));      // ipv6.rs:181-186
                ipid = ((b1 & 0x0F) << 16) | hb16(h, hl + 2);         // ipv6.rs:189-196
                iplen = (uint16_t)hb16(h, hl + 4);                    // ipv6.rs:199-202
            }
        } else {
            if (c.p[ZP_COL_SRC_ADDR]) ((uint4*)c.p[ZP_COL_SRC_ADDR])[i] = z;
            if (c.p[ZP_COL_DEST_ADDR]) ((uint4*)c.p[ZP_COL_DEST_ADDR])[i] = z;
        }
        if (r.flags & ZP_F_IP_IN_IP) {
            const bool v6 = (r.flags & ZP_F_IP_IN_IP_V6) != 0;
            const uint32_t p = r.inner_off;
            iv = (uint8_t)(hb(h, p) >> 4);
            st_addr(c, ZP_COL_INNER_SRC_ADDR, i, h, p + (v6 ? 8 : 12), v6);
            st_addr(c, ZP_COL_INNER_DEST_ADDR, i, h, p + (v6 ? 24 : 16), v6);
            iproto = v6 ? r.inner_final_nh : (uint8_t)hb(h, p + 9);
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
                sport = (uint16_t)hb16(h, p);                         // tcp.rs:151-154
                dport = (uint16_t)hb16(h, p + 2);                     // tcp.rs:157-160
                seq = hb32(h, p + 4);                                 // tcp.rs:163-170
                ack = hb32(h, p + 8);                                 // tcp.rs:172-179
                const uint32_t b12 = hb16(h, p + 12);
                tflags = (uint8_t)(b12 & 0xFF);                       // tcp.rs:193-196
                hlen = (b12 >> 12) * 4;                               // tcp.rs:217-220
                win16 = (uint16_t)hb16(h, p + 14);                    // tcp.rs:199-202
                l4ck = (uint16_t)hb16(h, p + 16);                     // tcp.rs:205-208
            } else if (l4f == ZP_F_UDP) {
                l4p = 17;
                sport = (uint16_t)hb16(h, p);                         // udp.rs:113-116
                dport = (uint16_t)hb16(h, p + 2);                     // udp.rs:119-122
                l4ck = (uint16_t)hb16(h, p + 6);                      // udp.rs:125-128
            } else {
                l4p = l4f == ZP_F_ICMPV4 ? 1 : 58;
                const uint32_t tc = hb16(h, p);
                ity = (uint8_t)(tc >> 8);                             // icmpv4.rs:102-105
                icode = (uint8_t)(tc & 0xFF);                         // icmpv4.rs:108-111
                l4ck = (uint16_t)hb16(h, p + 2);                      // icmpv4.rs:114-117
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

extern "C" int zp_extract_columns_device(const uint8_t* arena, const uint64_t* offs,
                                         const uint32_t* lens, const zp_record* records,
                                         uint64_t n, void* const* cols, void* stream) {
    if (n == 0) return 0;
    if (!arena || !offs || !lens || !records || !cols) {
        snprintf(zp__errbuf(), 256, "zp_extract_columns_device: null pointer");
        return -1;
    }
    ColPtrs c;
    bool any = false;
    for (int k = 0; k < ZP_COL_COUNT; ++k) {
        c.p[k] = (uint8_t*)cols[k];
        any |= c.p[k] != nullptr;
    }
    if (!any) return 0;
    const uint64_t blocks = (n + FX_BLOCK - 1) / FX_BLOCK;
    if (blocks > 0x7FFFFFFFull) {
        snprintf(zp__errbuf(), 256, "zp_extract_columns_device: batch too large");
        return -1;
    }
    hipLaunchKernelGGL(zp_columns_kernel, dim3((unsigned)blocks), dim3(FX_BLOCK), 0,
                       (hipStream_t)stream, arena, offs, lens, records, n, c);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        snprintf(zp__errbuf(), 256, "zp_columns_kernel launch: %s", hipGetErrorString(e));
        return -2;
    }
    return 0;
}
