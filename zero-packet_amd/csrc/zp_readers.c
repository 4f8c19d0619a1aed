/*
 * zp_readers.c — the standalone reader constructors and the checksum
 * primitives of the C ABI (include/zero_packet.h):
 *
 *   zp_reader_new               XReader::new(&[u8]) -> Result<Self, &'static str>
 *                               for the twelve reader views (README.md:110-115)
 *   zp_internet_checksum        internet_checksum          (checksum.rs:5-29)
 *   zp_verify_internet_checksum verify_internet_checksum   (checksum.rs:33-35)
 *   zp_pseudo_header            pseudo_header              (checksum.rs:38-69)
 *   zp_rec_decode               a zp_record unpacked (both forms, include/zero_packet.h)
 *
 * These are host functions over one host slice, as in the reference: a
 * reader is a view, its constructor checks a minimum length (Ethernet also
 * its VLAN tagging, IPv6 also runs the extension-header walk). The batch
 * parse of many frames is the device path (zp_parse.hip); nothing here
 * parses a frame.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/zero_packet.h"

static inline uint32_t be16_at(const uint8_t* p) { return ((uint32_t)p[0] << 8) | p[1]; }

/* checksum.rs:5-29. The reference adds into a u32 that wraps (release
 * build); a wrapping sum equals the exact sum mod 2^32, so the words are
 * summed exactly in 64 bits (vectorisable) and truncated once. */
uint16_t zp_internet_checksum(const uint8_t* data, uint64_t len, uint32_t accumulator) {
    uint64_t s = accumulator;
    const uint64_t even = len & ~(uint64_t)1;
    for (uint64_t i = 0; i < even; i += 2) s += be16_at(data + i);   /* :11-15 */
    if (len & 1) s += (uint32_t)data[len - 1] << 8;                  /* :18-20 */
    uint32_t sum = (uint32_t)s;
    while (sum >> 16) sum = (sum & 0xFFFFu) + (sum >> 16);           /* :23-25 */
    return (uint16_t)~sum;                                           /* :28 */
}

int zp_verify_internet_checksum(const uint8_t* data, uint64_t len, uint32_t accumulator) {
    return zp_internet_checksum(data, len, accumulator) == 0;
}

/* checksum.rs:43-69: PseudoHeader::sum of [u8; 4] / [u8; 16], plus the
 * protocol and `length as u32`. */
uint32_t zp_pseudo_header(const uint8_t* src, const uint8_t* dest, uint32_t addr_len,
                          uint8_t protocol, uint64_t length) {
    if ((addr_len != 4 && addr_len != 16) || !src || !dest) return 0;
    uint32_t s = 0;
    for (uint32_t k = 0; k < addr_len; k += 2) s += be16_at(src + k) + be16_at(dest + k);
    return s + protocol + (uint32_t)length;
}

/* ExtensionHeaders::parse (headers.rs:51-69) over the IPv6 payload `p`
 * (n bytes) starting with next header `nh`. Slot k's offset is relative to
 * the payload start. Returns ZP_OK or the first Err. */
static int ext_walk(const uint8_t* p, uint64_t n, uint8_t nh, zp_reader_info* info) {
    uint32_t have = 0;                  /* slots present, bit k = slot k */
    uint64_t at = 0;                    /* start of the current header  */
    uint32_t total = 0;
    uint8_t final_nh = 0;
    for (;;) {
        int slot;
        uint64_t min_len;
        int err_short, err_exceeds;
        if (nh == 0) {                                           /* :90-113 */
            if (have & (1u << ZP_EXT_HBH)) break;
            if (have) return ZP_ERR_EXT_HBH_NOT_FIRST;
            slot = ZP_EXT_HBH; min_len = 8;
            err_short = ZP_ERR_EXT_OPTIONS_TOO_SHORT; err_exceeds = ZP_ERR_EXT_OPTIONS_EXCEEDS;
        } else if (nh == 43) {                                   /* :117-134 */
            if (have & (1u << ZP_EXT_RT)) break;
            slot = ZP_EXT_RT; min_len = 8;
            err_short = ZP_ERR_EXT_ROUTING_TOO_SHORT; err_exceeds = ZP_ERR_EXT_ROUTING_EXCEEDS;
        } else if (nh == 44) {                                   /* :138-155 */
            if (have & (1u << ZP_EXT_FRAG)) break;
            slot = ZP_EXT_FRAG; min_len = 8;
            err_short = ZP_ERR_EXT_FRAGMENT_TOO_SHORT; err_exceeds = ZP_OK;
        } else if (nh == 51) {                                   /* :159-176 */
            if (have & (1u << ZP_EXT_AH)) break;
            slot = ZP_EXT_AH; min_len = 12;
            err_short = ZP_ERR_EXT_AUTH_TOO_SHORT; err_exceeds = ZP_ERR_EXT_AUTH_EXCEEDS;
        } else if (nh == 60) {                                   /* :180-202 */
            if (have & (1u << ZP_EXT_DST2)) break;
            slot = (have & (1u << ZP_EXT_DST1)) ? ZP_EXT_DST2 : ZP_EXT_DST1; min_len = 8;
            err_short = ZP_ERR_EXT_OPTIONS_TOO_SHORT; err_exceeds = ZP_ERR_EXT_OPTIONS_EXCEEDS;
        } else {
            break;                                               /* :84 */
        }
        const uint64_t left = n - at;
        if (left < min_len) return err_short;                    /* XReader::new */
        const uint8_t* h = p + at;
        const uint64_t hl = slot == ZP_EXT_FRAG ? 8                               /* fragment.rs:160 */
                          : slot == ZP_EXT_AH ? ((uint64_t)h[1] + 2) * 4           /* authentication.rs:178 */
                          : ((uint64_t)h[1] + 1) * 8;                              /* options.rs:127, routing.rs:172 */
        if (err_exceeds != ZP_OK && hl > left) return err_exceeds;                 /* payload()? */
        have |= 1u << slot;
        info->ext.off[slot] = (uint16_t)at;
        total += (uint32_t)hl;
        final_nh = h[0];
        nh = h[0];
        at += hl;
    }
    if (have) {                                                  /* :64-68 */
        info->flags = ZP_F_EXT;
        for (int k = 0; k < ZP_EXT_SLOTS; ++k)
            if (have & (1u << k)) info->flags |= ZP_F_EXT_SLOT(k);
        info->ext.len = (uint16_t)total;
        info->ext.final_nh = final_nh;                           /* headers.rs:26 */
        info->final_nh = final_nh;
    }
    return ZP_OK;
}

int zp_reader_new(int kind, const uint8_t* bytes, uint64_t len, zp_reader_info* info) {
    zp_reader_info local;
    if (!info) info = &local;
    memset(info, 0, sizeof *info);
    if (kind < 0 || kind >= ZP_READER_KIND_COUNT || (!bytes && len)) return -1;
    switch (kind) {
    case ZP_READER_ETHERNET: {                                   /* ethernet.rs:141-179 */
        if (len < 14) return ZP_ERR_ETH_SLICE_TOO_SHORT;
        const uint32_t t = be16_at(bytes + 12);
        if (t == 0x8100) {
            if (len < 18) return ZP_ERR_ETH_VLAN_TOO_SHORT;
            info->header_len = 18;
        } else if (t == 0x88A8) {
            if (len < 22) return ZP_ERR_ETH_QINQ_TOO_SHORT;
            if (be16_at(bytes + 16) != 0x8100) return ZP_ERR_ETH_INVALID_QINQ;
            info->header_len = 22;
        } else {
            info->header_len = 14;
        }
        return ZP_OK;
    }
    case ZP_READER_ARP:      return len < 28 ? ZP_ERR_ARP_TOO_SHORT : ZP_OK;          /* arp.rs:131 */
    case ZP_READER_IPV4:     return len < 20 ? ZP_ERR_IPV4_TOO_SHORT : ZP_OK;         /* ipv4.rs:139 */
    case ZP_READER_IPV6: {                                                            /* ipv6.rs:147-167 */
        if (len < 40) return ZP_ERR_IPV6_TOO_SHORT;
        const int e = ext_walk(bytes + 40, len - 40, bytes[6], info);  /* :159, before any */
        if (e != ZP_OK) {                                               /* version check   */
            memset(info, 0, sizeof *info);
            return e;
        }
        if (!(info->flags & ZP_F_EXT)) info->final_nh = bytes[6];     /* ipv6.rs:219-227 */
        return ZP_OK;
    }
    case ZP_READER_OPTIONS:  return len < 8 ? ZP_ERR_EXT_OPTIONS_TOO_SHORT : ZP_OK;   /* options.rs:84 */
    case ZP_READER_ROUTING:  return len < 8 ? ZP_ERR_EXT_ROUTING_TOO_SHORT : ZP_OK;   /* routing.rs:108 */
    case ZP_READER_FRAGMENT: return len < 8 ? ZP_ERR_EXT_FRAGMENT_TOO_SHORT : ZP_OK;  /* fragment.rs:98 */
    case ZP_READER_AUTH:     return len < 12 ? ZP_ERR_EXT_AUTH_TOO_SHORT : ZP_OK;     /* authentication.rs:106 */
    case ZP_READER_TCP:      return len < 20 ? ZP_ERR_TCP_TOO_SHORT : ZP_OK;          /* tcp.rs:142 */
    case ZP_READER_UDP:      return len < 8 ? ZP_ERR_UDP_TOO_SHORT : ZP_OK;           /* udp.rs:104 */
    case ZP_READER_ICMPV4:   return len < 8 ? ZP_ERR_ICMP_TOO_SHORT : ZP_OK;          /* icmpv4.rs:93 */
    case ZP_READER_ICMPV6:   return len < 8 ? ZP_ERR_ICMP_TOO_SHORT : ZP_OK;          /* icmpv6.rs:90 */
    }
    return -1;
}

/* IPv6 header at frame[ip..]: its extension chain's length and
 * final_next_header (ipv6.rs:141, :219-227), from the caller's entry when it
 * has one, else by the walk IPv6Reader::new runs (ipv6.rs:159). */
static int ipv6_chain(const uint8_t* frame, uint64_t len, uint64_t ip, int chained,
                      const zp_ext_offsets* x, uint32_t* chain_len, uint8_t* final_nh) {
    if (ip + 40 > len) return -1;
    if (!chained) {
        *chain_len = 0;
        *final_nh = frame[ip + 6];
        return 0;
    }
    if (x) {
        *chain_len = x->len;
        *final_nh = x->final_nh;
        return 0;
    }
    zp_reader_info info;
    if (zp_reader_new(ZP_READER_IPV6, frame + ip, len - ip, &info) != ZP_OK ||
        !(info.flags & ZP_F_EXT))
        return -1;
    *chain_len = info.ext.len;
    *final_nh = info.final_nh;
    return 0;
}

int zp_rec_decode(const zp_record* rec, const uint8_t* frame, uint64_t len,
                  const zp_ext_offsets* ext, zp_rec_fields* out) {
    if (!rec || !out || (!frame && len)) return -1;
    memset(out, 0, sizeof *out);
    const zp_record r = *rec;
    out->err = (uint8_t)zp_rec_err(r);
    if (out->err) return 0;                         /* Err: no readers */
    const uint32_t flags = r.flags & ZP_F_MASK;
    out->flags = flags;
    out->l4_off = zp_rec_l4_off(r);
    const uint32_t l4_any = ZP_F_TCP | ZP_F_UDP | ZP_F_ICMPV4 | ZP_F_ICMPV6;
    uint32_t outer_chain = 0;
    if (zp_rec_is_far(r)) {
        zp_reader_info eth;
        if (!(flags & l4_any) || !(flags & ZP_F_IP_IN_IP) ||
            zp_reader_new(ZP_READER_ETHERNET, frame, len, &eth) != ZP_OK)
            return -1;
        out->eth_len = (uint8_t)eth.header_len;                  /* ethernet.rs:155-179 */
    } else {
        out->eth_len = (uint8_t)zp_rec_eth_len(r);
        out->inner_off = zp_rec_inner_off(r);
    }
    const uint64_t hl = out->eth_len;
    if (flags & ZP_F_IPV6) {
        zp_ext_offsets inl;
        const int il = zp_rec_chain_inline(r);                    /* ABI v6 */
        if (il) zp_rec_chain(r, &inl);
        if (ipv6_chain(frame, len, hl, (flags & ZP_F_EXT) != 0, il ? &inl : ext ? &ext[0] : NULL,
                       &outer_chain, &out->final_nh))
            return -1;
    }
    if (zp_rec_is_far(r)) {
        /* the ip_in_ip header follows the outer IP header (parser.rs:134-135) */
        if (flags & ZP_F_IPV4) {
            if (hl >= len) return -1;
            out->inner_off = (uint32_t)hl + (frame[hl] & 15u) * 4u;   /* ipv4.rs:228-258 */
        } else if (flags & ZP_F_IPV6) {
            out->inner_off = (uint32_t)hl + 40u + outer_chain;         /* ipv6.rs:283-285 */
        } else {
            return -1;
        }
    }
    if ((flags & ZP_F_IP_IN_IP_V6) &&
        ipv6_chain(frame, len, out->inner_off, (flags & ZP_F_INNER_EXT) != 0,
                   ext ? &ext[1] : NULL, &outer_chain, &out->inner_final_nh))
        return -1;
    if ((flags & ZP_F_IP_IN_IP) && out->inner_off >= len) return -1;
    if ((flags & l4_any) && out->l4_off >= len) return -1;
    return 0;
}
