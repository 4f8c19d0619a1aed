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
#include "zp_cols.h"

extern "C" char* zp__errbuf(void);

#ifndef FX_WIN
#define FX_WIN 112                       // staged bytes per frame (from A & ~15); longer headers
                                         // (some c4 chains) read the rest from HBM. 112 vs 160:
                                         // c3 -5 %, c5 -9 %, c4 +-2 % (28 KB of LDS per workgroup
                                         // instead of 40: more workgroups per CU; r04_cols_window_ab.log)
#endif
#define FX_CH (FX_WIN / 16)
#define FX_BLOCK 256

static const int kColWidth[ZP_COL_COUNT] = {
    6, 6, 2, 2, 2, 2, 1, 16, 16, 1, 1, 1, 4, 2, 1, 16, 16, 1, 1, 2, 2, 4, 4, 1, 2, 1, 1, 2, 4};

extern "C" int zp_col_width(int col) {
    return col >= 0 && col < ZP_COL_COUNT ? kColWidth[col] : 0;
}

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
    // byte y & 15 of the chunk by shifts and one select (a select chain over
    // the four dwords was lowered to a dynamically indexed scratch copy)
    const uint64_t q = (y & 8) ? (((uint64_t)h.xc.w << 32) | h.xc.z)
                               : (((uint64_t)h.xc.y << 32) | h.xc.x);
    return (uint32_t)(q >> (8 * (y & 7))) & 0xFFu;
}
// Dword z (4-aligned, from A & ~15) of the staged window.
__device__ __forceinline__ uint32_t hdw(const Hdr& h, uint32_t z) {
    return *(const uint32_t*)(h.win + (z >> 4) * 16 * FX_BLOCK + (z & 15));
}
struct HdrReader {
    Hdr& h;
    __device__ __forceinline__ uint32_t operator()(uint32_t x) { return hb(h, x); }
    __device__ __forceinline__ bool has4(uint32_t x) const { return x + 3 < h.wlen; }
    __device__ __forceinline__ uint32_t le4(uint32_t x) const {
        const uint32_t y = x + h.shift, z = y & ~3u;
        const uint32_t lo = hdw(h, z), hi = (y & 3) ? hdw(h, z + 4) : 0u;
        return __builtin_amdgcn_alignbyte(hi, lo, y & 3);
    }
};

// IPv6Reader::final_next_header (ipv6.rs:219-227) of the IPv6 header at
// `ip`: its next-header byte, or with an extension chain the next-header
// byte of the chain's last header (headers.rs:51-213 stops after the
// headers the slot bits name; lengths by type as in the walk).
// *end = the upper-layer payload's start (ipv6.rs:283-285).
template <class R>
__device__ __forceinline__ uint32_t final_nh(R& rd, uint32_t ip, uint32_t slots, uint32_t* end) {
    uint32_t cur = rd(ip + 6), p = ip + 40;
    for (int k = __builtin_popcount(slots & 63u); k > 0; --k) {
        const uint32_t b1 = rd(p + 1);
        const uint32_t hl = cur == 44 ? 8u : cur == 51 ? (b1 + 2) * 4 : (b1 + 1) * 8;
        cur = rd(p);
        p += hl;
    }
    *end = p;
    return cur;
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
    // the 8-B record, unpacked (include/zero_packet.h); the final next
    // headers of the IPv6 readers come from the frame after the staging
    zp_rec_full r;
    static_assert(sizeof(zp_record) == 8, "one 8-B load per record");
    const zp_u32x2 q = *(const FX_GLOBAL zp_u32x2*)(recs + i);
    r.flags = q.x & ZP_F_MASK;
    r.err = (uint8_t)(q.x >> 26);
    r.final_nh = 0;
    r.inner_final_nh = 0;
    // The far-L4 form (an L4 reader past byte 262,143): offs holds the whole
    // L4 offset; the Ethernet header length and inner_off are read from the
    // frame after the staging (include/zero_packet.h).
    const bool far = ((q.x >> 24) & 3u) == ZP_ETH_CODE_FAR;
    r.eth_len = (uint8_t)(far ? 22u : 14u + 4u * ((q.x >> 24) & 3u));
    r.l4_off = far ? q.y : q.y & ZP_L4_NEAR_MAX;
    r.inner_off = far || !(r.flags & ZP_F_IP_IN_IP) ? 0u : q.y >> 18;   // else: an inline chain
    r.chain = 0;
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
    if (far) need = FX_WIN;             // eth_len / inner_off not known yet
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
            const uint32_t f = 8 * q + (lane >> 3);
            const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(f << 2), (int)a_lo);
            const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(f << 2), (int)a_hi);
            const uint32_t nc = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(f << 2), (int)nch);
            // windows past 128 B: further rounds of 8 chunks per frame
#pragma unroll
            for (uint32_t g = 0; g < (FX_CH + 7) / 8; ++g) {
                const uint32_t ch = 8 * g + (lane & 7);
                if (ch < nc && ch < FX_CH)
                    win[ch * FX_BLOCK + wbase + f] =
                        fx_ld16((((uintptr_t)hi << 32) | lo) + 16u * ch);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }

    if (!live) return;
    HdrReader rd{h};
    if (ok && far) {
        const uint32_t t0 = rd16(rd, 12u);                          // ethernet.rs:155-179
        r.eth_len = (uint8_t)(t0 == 0x8100 ? 18u : t0 == 0x88A8 ? 22u : 14u);
    }
    uint32_t ulp = 0;
    if (ok && (r.flags & ZP_F_IPV6))
        r.final_nh = (uint8_t)final_nh(rd, r.eth_len, r.flags >> 12, &ulp);
    if (ok && far)                      // ip_in_ip follows the outer IP header
        r.inner_off = (r.flags & ZP_F_IPV6) ? ulp : r.eth_len + (rd(r.eth_len) & 15u) * 4u;
    if (ok && (r.flags & ZP_F_IP_IN_IP_V6))
        r.inner_final_nh = (uint8_t)final_nh(rd, r.inner_off, r.flags >> 18, &ulp);
    emit_columns(rd, r, ok, len, i, c);
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
