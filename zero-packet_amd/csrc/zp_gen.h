/*
 * zp_gen.h — deterministic synthetic frame generator for the BASELINE.json
 * configs. Header-only; compiled into the HIP library
 * (device kernels, zp_gen.hip) and into the host library (zp_host.c), so
 * GPU- and CPU-generated batches are byte-identical by construction.
 *
 * Frame content follows the reference builder's field layout and
 * checksum-fill semantics:
 *   - Ethernet / VLAN / Q-in-Q writers     ethernet.rs:45-128
 *   - IPv4 writer + header checksum        ipv4.rs:33-126 (set_checksum :119)
 *   - IPv6 writer                          ipv6.rs:30-132
 *   - Options / Routing / Fragment writers options.rs:6-74, routing.rs:6-97,
 *                                          fragment.rs:6-88
 *   - TCP / UDP / ICMP checksum over the whole remaining segment with the
 *     pseudo-header sum (builder.rs:473-474, 515-516, 553, 592-593;
 *     tcp.rs:123-129, udp.rs:65-71, icmpv4.rs:74-80, icmpv6.rs:71-77).
 * Every generated frame is accepted by PacketParser::parse; the tests check
 * that against the oracle.
 *
 * Packet i of (config, seed) depends only on (config, seed, i):
 * key = splitmix64(seed ^ i * 0x9E3779B97F4A7C15).
 */
#ifndef ZP_GEN_H
#define ZP_GEN_H

#include <stdint.h>

#if defined(__HIPCC__)
#define ZP_HD __host__ __device__ __forceinline__
#else
#define ZP_HD static inline
#endif

#define ZP_GOLDEN 0x9E3779B97F4A7C15ull

ZP_HD uint64_t zp_mix64(uint64_t z) {
    z += ZP_GOLDEN;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Field hash: independent 64-bit value per (packet key, salt). */
ZP_HD uint64_t zp_h(uint64_t key, uint64_t salt) {
    return zp_mix64(key ^ (salt * 0xD1B54A32D192ED03ull));
}

/* Uniform integer in [0, m) from a 64-bit hash (m < 2^32). */
ZP_HD uint32_t zp_below(uint64_t h, uint32_t m) {
    return (uint32_t)(((h >> 32) * (uint64_t)m) >> 32);
}

/* Valid ICMPv4 types (misc.rs:93-119) and ICMPv6 types (misc.rs:164-204). */
ZP_HD uint8_t zp_icmpv4_type_at(uint32_t i) {
    const uint8_t t[21] = {0, 3, 4, 5, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18,
                           30, 40, 42, 43, 253, 254};
    return t[i % 21];
}
ZP_HD uint8_t zp_icmpv6_type_at(uint32_t i) {
    const uint8_t t[35] = {1, 2, 3, 4, 100, 101, 128, 129, 130, 131, 132, 133,
                           134, 135, 136, 137, 138, 139, 140, 141, 142, 143,
                           144, 145, 146, 147, 148, 149, 150, 151, 152, 153,
                           155, 200, 201};
    return t[i % 35];
}

/* Salts for field hashes. */
enum {
    ZP_S_LEN = 1, ZP_S_VLAN, ZP_S_OUTER, ZP_S_INNER, ZP_S_L4, ZP_S_EXT,
    ZP_S_HBH, ZP_S_RT, ZP_S_DOFF, ZP_S_ICMP, ZP_S_MAC, ZP_S_TCI,
    ZP_S_IP4O, ZP_S_IP4I, ZP_S_IP6O, ZP_S_IP6I, ZP_S_L4F, ZP_S_PAY,
    ZP_S_EXTDATA, ZP_S_FLAGS, ZP_S_MIX, ZP_S_ARP
};

typedef struct zp_plan {
    uint64_t key;
    uint32_t len;          /* frame length                                   */
    uint16_t eth_len;      /* 14 / 18 / 22                                   */
    uint16_t ext_len;      /* outer IPv6 extension bytes                     */
    uint16_t inner_off;    /* 0 if no IP-in-IP                               */
    uint16_t l4_off;
    uint16_t l4_hdr;       /* L4 header bytes (TCP doff*4, else 8)           */
    uint16_t pay_off;      /* first payload byte                             */
    uint8_t  vlan;         /* 0 none, 1 802.1Q, 2 Q-in-Q                     */
    uint8_t  outer;        /* 4 or 6; 0 = ARP (config 6)                     */
    uint8_t  inner;        /* 0, 4 or 6                                      */
    uint8_t  l4;           /* 6 TCP, 17 UDP, 1 ICMPv4, 58 ICMPv6             */
    uint8_t  ext_mask;     /* outer IPv6: 1 HBH, 2 Routing, 4 Fragment       */
    uint8_t  hbh_el, rt_el;/* header ext len fields                          */
    uint8_t  tcp_doff;
    uint8_t  icmp_type, icmp_code, tcp_flags;
    uint16_t csum_o4, csum_i4, csum_l4;  /* checksum field values            */
} zp_plan;

ZP_HD uint32_t zp_ip_hdr_len(uint8_t v) { return v == 4 ? 20u : (v == 6 ? 40u : 0u); }

/* Lays out a header stack and returns its byte size. */
ZP_HD uint32_t zp_plan_layout(zp_plan* p) {
    uint32_t pos = p->eth_len;
    uint32_t ext = 0;
    if (p->outer == 0) {           /* ARP: 28-B header, then padding (arp.rs:121-176) */
        p->ext_len = 0; p->inner_off = 0; p->l4_hdr = 0;
        p->l4_off = p->pay_off = (uint16_t)(pos + 28u);
        return pos + 28u;
    }
    if (p->outer == 6) {
        if (p->ext_mask & 1) ext += ((uint32_t)p->hbh_el + 1u) * 8u;
        if (p->ext_mask & 2) ext += ((uint32_t)p->rt_el + 1u) * 8u;
        if (p->ext_mask & 4) ext += 8u;
    }
    p->ext_len = (uint16_t)ext;
    pos += zp_ip_hdr_len(p->outer) + ext;
    p->inner_off = (uint16_t)(p->inner ? pos : 0);
    pos += zp_ip_hdr_len(p->inner);
    p->l4_off = (uint16_t)pos;
    p->l4_hdr = (uint16_t)(p->l4 == 6 ? (uint32_t)p->tcp_doff * 4u : 8u);
    pos += p->l4_hdr;
    p->pay_off = (uint16_t)pos;
    return pos;
}

/* IMIX size for C5: {64, 576, 1500} with weights 7:4:1. */
ZP_HD uint32_t zp_imix_len(uint64_t h) {
    uint32_t r = zp_below(h, 12);
    return r < 7 ? 64u : (r < 11 ? 576u : 1500u);
}

/* Config 6 (mixed traffic, no BASELINE counterpart): each packet takes the
 * shape of config 3, 4 or 5 (5/16 each) or is an ARP request / reply (1/16,
 * 64 B, any tagging), so every 64-frame tile mixes all header stacks. */
ZP_HD int zp_mix_shape(uint64_t key) {
    const uint32_t r = zp_below(zp_h(key, ZP_S_MIX), 16);
    return r == 0 ? 0 : (r <= 5 ? 3 : (r <= 10 ? 4 : 5));
}

/* Draws the structure of packet `idx` (everything except checksums). */
ZP_HD void zp_plan_packet(int cfg, uint64_t seed, uint64_t idx, zp_plan* p) {
    const uint64_t key = zp_mix64(seed ^ (idx * ZP_GOLDEN));
    p->key = key;
    p->vlan = 0; p->outer = 4; p->inner = 0; p->l4 = 17; p->ext_mask = 0;
    p->hbh_el = 0; p->rt_el = 0; p->tcp_doff = 5; p->icmp_type = 0;
    p->icmp_code = 0; p->csum_o4 = 0; p->csum_i4 = 0; p->csum_l4 = 0;
    p->tcp_flags = (uint8_t)(1u + zp_below(zp_h(key, ZP_S_FLAGS), 255));
    uint32_t len = 64;
    if (cfg == 6) {
        cfg = zp_mix_shape(key);
        if (cfg == 0) {                   /* ARP */
            p->outer = 0; p->l4 = 0;
            p->vlan = (uint8_t)zp_below(zp_h(key, ZP_S_VLAN), 3);
            p->eth_len = (uint16_t)(14u + 4u * p->vlan);
            zp_plan_layout(p);
            p->len = 64;
            return;
        }
    }
    if (cfg == 3) {                       /* IPv4, TCP/UDP/ICMPv4, U[64,1500] */
        len = 64u + zp_below(zp_h(key, ZP_S_LEN), 1437);
        uint32_t l4 = zp_below(zp_h(key, ZP_S_L4), 3);
        p->l4 = l4 == 0 ? 6 : (l4 == 1 ? 17 : 1);
    } else if (cfg == 4) {                /* IPv6 + ext chain + VLAN/QinQ     */
        p->outer = 6;
        p->vlan = (uint8_t)zp_below(zp_h(key, ZP_S_VLAN), 3);
        p->ext_mask = (uint8_t)zp_below(zp_h(key, ZP_S_EXT), 8);
        p->hbh_el = (uint8_t)zp_below(zp_h(key, ZP_S_HBH), 3);
        p->rt_el = (uint8_t)zp_below(zp_h(key, ZP_S_RT), 5);
        uint32_t l4 = zp_below(zp_h(key, ZP_S_L4), 3);
        p->l4 = l4 == 0 ? 6 : (l4 == 1 ? 17 : 58);
    } else if (cfg == 5) {                /* IMIX, v4/v6, 25 % IP-in-IP       */
        len = zp_imix_len(zp_h(key, ZP_S_LEN));
        p->vlan = (uint8_t)zp_below(zp_h(key, ZP_S_VLAN), 3);
        p->outer = zp_below(zp_h(key, ZP_S_OUTER), 2) ? 6 : 4;
        uint32_t enc = zp_below(zp_h(key, ZP_S_INNER), 8);
        p->inner = enc < 6 ? 0 : (enc == 6 ? 4 : 6);
        uint32_t l4 = zp_below(zp_h(key, ZP_S_L4), 3);
        uint8_t innermost = p->inner ? p->inner : p->outer;
        p->l4 = l4 == 0 ? 6 : (l4 == 1 ? 17 : (innermost == 4 ? 1 : 58));
    }
    if (p->l4 == 6) p->tcp_doff = (uint8_t)(5u + zp_below(zp_h(key, ZP_S_DOFF), 4));
    p->eth_len = (uint16_t)(14u + 4u * p->vlan);
    uint32_t hdr = zp_plan_layout(p);
    if (cfg == 5) {
        /* Header stacks are drawn from those that fit the drawn size:
         * shrink TCP options, drop VLAN tags, fall back to UDP, and drop
         * the encapsulation last. */
        if (hdr > len && p->l4 == 6) { p->tcp_doff = 5; hdr = zp_plan_layout(p); }
        if (hdr > len && p->vlan) { p->vlan = 0; p->eth_len = 14; hdr = zp_plan_layout(p); }
        if (hdr > len) { p->l4 = 17; hdr = zp_plan_layout(p); }
        if (hdr > len && p->inner) { p->inner = 0; hdr = zp_plan_layout(p); }
    } else if (cfg == 3) {
        if (hdr > len) {   /* TCP doff must leave room in a short frame */
            p->tcp_doff = (uint8_t)((len - 34u) / 4u);
            if (p->tcp_doff > 8) p->tcp_doff = 8;
            hdr = zp_plan_layout(p);
        }
    } else if (cfg == 4) {
        uint32_t lo = hdr > 64u ? hdr : 64u;
        len = lo + zp_below(zp_h(key, ZP_S_LEN), 1501u - lo);
    }
    if (p->l4 == 1 || p->l4 == 58) {
        uint32_t h = (uint32_t)zp_h(key, ZP_S_ICMP);
        p->icmp_type = p->l4 == 1 ? zp_icmpv4_type_at(h & 0xFFFF) : zp_icmpv6_type_at(h & 0xFFFF);
        p->icmp_code = p->l4 == 1 ? (uint8_t)((h >> 16) % 16u) : (uint8_t)(h >> 24);
    }
    p->len = len;
}

/* Next-header value that follows the outer IPv6 extension slot `slot`
 * (0 = the IPv6 header itself, then HBH, Routing, Fragment in RFC order). */
ZP_HD uint8_t zp_after_ext(const zp_plan* p, int slot) {
    for (int s = slot; s < 3; ++s)
        if (p->ext_mask & (1 << s)) return (uint8_t)(s == 0 ? 0 : (s == 1 ? 43 : 44));
    if (p->inner) return (uint8_t)(p->inner == 4 ? 4 : 41);
    return p->l4;
}

ZP_HD uint8_t zp_hbyte(uint64_t key, uint64_t salt, uint32_t i) {
    return (uint8_t)(zp_h(key, salt + 64u * (i >> 3)) >> (8u * (i & 7u)));
}

/* IPv4 header byte x of a header at frame offset `base`. */
ZP_HD uint8_t zp_ip4_byte(const zp_plan* p, uint32_t base, uint32_t x,
                          uint8_t proto, uint16_t csum, uint64_t salt) {
    switch (x) {
    case 0: return 0x45;
    case 1: return zp_hbyte(p->key, salt, 0) & 0xFC;
    case 2: return (uint8_t)((p->len - base) >> 8);
    case 3: return (uint8_t)(p->len - base);
    case 4: return zp_hbyte(p->key, salt, 1);
    case 5: return zp_hbyte(p->key, salt, 2);
    case 6: return 0x40;                /* DF */
    case 7: return 0;
    case 8: return 64;
    case 9: return proto;
    case 10: return (uint8_t)(csum >> 8);
    case 11: return (uint8_t)csum;
    default: return zp_hbyte(p->key, salt, 4 + x);   /* src / dst */
    }
}

/* IPv6 header byte x of a header at frame offset `base`. */
ZP_HD uint8_t zp_ip6_byte(const zp_plan* p, uint32_t base, uint32_t x,
                          uint8_t nh, uint64_t salt) {
    uint32_t tc = zp_hbyte(p->key, salt, 0);
    uint32_t fl = (uint32_t)(zp_h(p->key, salt + 1000) & 0xFFFFF);
    uint32_t plen = p->len - base - 40u;
    switch (x) {
    case 0: return (uint8_t)(0x60 | (tc >> 4));
    case 1: return (uint8_t)(((tc & 15) << 4) | (fl >> 16));
    case 2: return (uint8_t)(fl >> 8);
    case 3: return (uint8_t)fl;
    case 4: return (uint8_t)(plen >> 8);
    case 5: return (uint8_t)plen;
    case 6: return nh;
    case 7: return 64;
    default: return zp_hbyte(p->key, salt, 8 + x);   /* src / dst */
    }
}

/* Byte `pos` of the frame (pos < p->len). */
ZP_HD uint8_t zp_gen_byte(const zp_plan* p, uint32_t pos) {
    const uint64_t key = p->key;
    if (pos < p->eth_len) {
        if (pos < 12) return zp_hbyte(key, ZP_S_MAC, pos);
        uint32_t ethertype = p->outer == 4 ? 0x0800u : (p->outer == 6 ? 0x86DDu : 0x0806u);
        uint32_t w;   /* 16-bit word at [pos & ~1] */
        uint32_t x = pos - 12;
        if (p->vlan == 0) w = ethertype;
        else if (p->vlan == 1) w = x < 2 ? 0x8100u : (x < 4 ? (uint32_t)(zp_h(key, ZP_S_TCI) & 0xFFF) : ethertype);
        else w = x < 2 ? 0x88A8u : (x < 4 ? (uint32_t)(zp_h(key, ZP_S_TCI) & 0xFFF)
                 : (x < 6 ? 0x8100u : (x < 8 ? (uint32_t)((zp_h(key, ZP_S_TCI) >> 16) & 0xFFF) : ethertype)));
        return (uint8_t)((x & 1) ? w : (w >> 8));
    }
    uint32_t l3 = p->eth_len;
    if (p->outer == 0) {                   /* ARP (arp.rs:130-227 getters) */
        if (pos < l3 + 28u) {
            const uint32_t x = pos - l3;
            if (x == 0 || x == 3) return 0;                     /* htype 1, ptype 0x0800 */
            if (x == 1) return 1;
            if (x == 2) return 8;
            if (x == 4) return 6;                               /* hlen */
            if (x == 5) return 4;                               /* plen */
            if (x == 6) return 0;
            if (x == 7) return (uint8_t)(1u + zp_below(zp_h(key, ZP_S_ARP), 2));  /* oper 1|2 */
            return zp_hbyte(key, ZP_S_ARP + 1, x);             /* sha spa tha tpa */
        }
        return zp_hbyte(key, ZP_S_PAY, pos - p->pay_off);
    }
    if (p->outer == 4) {
        if (pos < l3 + 20u)
            return zp_ip4_byte(p, l3, pos - l3, zp_after_ext(p, 0), p->csum_o4, ZP_S_IP4O);
    } else {
        if (pos < l3 + 40u)
            return zp_ip6_byte(p, l3, pos - l3, zp_after_ext(p, 0), ZP_S_IP6O);
        uint32_t e = l3 + 40u;
        if (p->ext_mask & 1) {
            uint32_t hl = ((uint32_t)p->hbh_el + 1u) * 8u;
            if (pos < e + hl) {
                uint32_t x = pos - e;
                return x == 0 ? zp_after_ext(p, 1) : (x == 1 ? p->hbh_el : 0);
            }
            e += hl;
        }
        if (p->ext_mask & 2) {
            uint32_t hl = ((uint32_t)p->rt_el + 1u) * 8u;
            if (pos < e + hl) {
                uint32_t x = pos - e;
                if (x == 0) return zp_after_ext(p, 2);
                if (x == 1) return p->rt_el;
                if (x == 2) return 4;                       /* Segment Routing */
                if (x == 3) return (uint8_t)(zp_hbyte(key, ZP_S_EXTDATA, 0) & 3);
                if (x < 8) return 0;
                return zp_hbyte(key, ZP_S_EXTDATA, x);
            }
            e += hl;
        }
        if (p->ext_mask & 4) {
            if (pos < e + 8u) {
                uint32_t x = pos - e;
                if (x == 0) return zp_after_ext(p, 3);
                if (x < 4) return 0;                        /* offset 0, M = 0 */
                return zp_hbyte(key, ZP_S_EXTDATA, 100 + x);
            }
        }
    }
    if (p->inner && pos < p->l4_off) {
        uint32_t x = pos - p->inner_off;
        if (p->inner == 4) return zp_ip4_byte(p, p->inner_off, x, p->l4, p->csum_i4, ZP_S_IP4I);
        return zp_ip6_byte(p, p->inner_off, x, p->l4, ZP_S_IP6I);
    }
    if (pos < p->pay_off) {
        uint32_t x = pos - p->l4_off;
        if (p->l4 == 6) {
            if (x == 12) return (uint8_t)(p->tcp_doff << 4);
            if (x == 13) return p->tcp_flags;
            if (x == 16) return (uint8_t)(p->csum_l4 >> 8);
            if (x == 17) return (uint8_t)p->csum_l4;
            if (x == 18 || x == 19) return 0;
            if (x >= 20) return 1;                          /* NOP options */
            return zp_hbyte(key, ZP_S_L4F, x);
        }
        if (p->l4 == 17) {
            if (x == 4) return (uint8_t)((p->len - p->l4_off) >> 8);
            if (x == 5) return (uint8_t)(p->len - p->l4_off);
            if (x == 6) return (uint8_t)(p->csum_l4 >> 8);
            if (x == 7) return (uint8_t)p->csum_l4;
            return zp_hbyte(key, ZP_S_L4F, x);
        }
        if (x == 0) return p->icmp_type;
        if (x == 1) return p->icmp_code;
        if (x == 2) return (uint8_t)(p->csum_l4 >> 8);
        if (x == 3) return (uint8_t)p->csum_l4;
        return zp_hbyte(key, ZP_S_L4F, x);
    }
    return zp_hbyte(key, ZP_S_PAY, pos - p->pay_off);
}

/* Reference internet checksum finish: fold, one's complement (checksum.rs:22-28). */
ZP_HD uint16_t zp_fold_not(uint32_t sum) {
    while (sum >> 16) sum = (sum & 0xFFFFu) + (sum >> 16);
    return (uint16_t)~sum;
}

/* Big-endian 16-bit word sum of frame bytes [lo, hi) in reference word
 * parity (word starts at lo), with checksum fields currently in the plan. */
ZP_HD uint32_t zp_gen_sum(const zp_plan* p, uint32_t lo, uint32_t hi) {
    uint32_t s = 0;
    for (uint32_t i = lo; i < hi; ++i)
        s += (uint32_t)zp_gen_byte(p, i) << (((i - lo) & 1u) ? 0 : 8);
    return s;
}

/* Pseudo-header sum of the innermost IP header for the L4 checksum
 * (checksum.rs:38-69; ICMPv4 under IPv4 uses no pseudo-header, parser.rs:322). */
ZP_HD uint32_t zp_gen_pseudo(const zp_plan* p) {
    uint8_t ip = p->inner ? p->inner : p->outer;
    if (ip == 0) return 0;                      /* ARP: no L4 */
    uint32_t base = p->inner ? p->inner_off : p->eth_len;
    uint32_t seglen = p->len - p->l4_off;
    if (ip == 4) {
        if (p->l4 == 1) return 0;
        return zp_gen_sum(p, base + 12, base + 20) + p->l4 + seglen;
    }
    return zp_gen_sum(p, base + 8, base + 40) + p->l4 + seglen;
}

/* Fills the IPv4 header checksums (header-only sums, independent of L4). */
ZP_HD void zp_plan_ip_csums(zp_plan* p) {
    p->csum_o4 = 0; p->csum_i4 = 0; p->csum_l4 = 0;
    if (p->outer == 4) p->csum_o4 = zp_fold_not(zp_gen_sum(p, p->eth_len, p->eth_len + 20u));
    if (p->inner == 4) p->csum_i4 = zp_fold_not(zp_gen_sum(p, p->inner_off, p->inner_off + 20u));
}

/* L4 checksum from the segment word sum computed with csum_l4 == 0. */
ZP_HD uint16_t zp_plan_l4_csum(const zp_plan* p, uint32_t seg_sum) {
    return zp_fold_not(zp_gen_pseudo(p) + seg_sum);
}

#endif /* ZP_GEN_H */
