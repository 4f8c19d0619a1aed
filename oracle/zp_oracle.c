/*
 * zp_oracle.c — CPU ORACLE for PacketParser::parse. TEST INFRASTRUCTURE ONLY.
 *
 * A scalar C restatement of the reference Rust parse path, written to mirror
 * its structure (readers over slices that run to the frame end, recursion for
 * IP-in-IP, byte-wise internet_checksum with u32 wrap-around). It is the
 * checker for the HIP path: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product (libzp_hip.so) never
 * links or calls it.
 *
 * Pinning: the reference is Rust and no Rust toolchain exists in this image
 * (SURVEY.md §8(c)), so it cannot be compiled or run here. This restatement
 * is pinned by the reference's own golden packets and known-answer tests
 * (parser.rs:369-959, builder.rs:1052-1296, checksum.rs:75-133), committed as
 * fixtures under tests/golden/ and checked by tests/test_oracle_golden.py.
 *
 * Each function cites the reference file:line it follows.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include "../include/zero_packet.h"

typedef struct { const uint8_t* p; size_t n; } slice_t;

static slice_t sub(slice_t s, size_t from) { slice_t r = {s.p + from, s.n - from}; return r; }
static uint16_t be16(slice_t s, size_t i) { return (uint16_t)((s.p[i] << 8) | s.p[i + 1]); }

/* ---- checksum.rs ------------------------------------------------------- */

/* checksum.rs:5-29. Rust release semantics: `sum +=` wraps at 2^32. */
uint16_t zpo_internet_checksum(const uint8_t* data, size_t len, uint32_t accumulator) {
    uint32_t sum = accumulator;
    size_t count = len, i = 0;
    while (count > 1) {                                   /* :11-15 */
        sum += ((uint32_t)data[i] << 8) | (uint32_t)data[i + 1];
        i += 2;
        count -= 2;
    }
    if (count > 0) sum += (uint32_t)data[i] << 8;         /* :18-20 */
    while (sum >> 16 != 0) sum = (sum & 0xFFFF) + (sum >> 16);   /* :23-25 */
    return (uint16_t)~sum;                                /* :28 */
}

/* checksum.rs:33-35 */
static int verify_internet_checksum(slice_t d, uint32_t acc) {
    return zpo_internet_checksum(d.p, d.n, acc) == 0;
}

/* checksum.rs:43-69 (PseudoHeader for [u8;4] / [u8;16], pseudo_header). */
uint32_t zpo_pseudo_header(const uint8_t* src, const uint8_t* dst, size_t addr_len,
                           uint8_t protocol, size_t length) {
    uint32_t s = 0;
    for (size_t k = 0; k < addr_len; k += 2) s += ((uint32_t)src[k] << 8) | src[k + 1];
    for (size_t k = 0; k < addr_len; k += 2) s += ((uint32_t)dst[k] << 8) | dst[k + 1];
    return s + protocol + (uint32_t)length;
}

/* ---- misc.rs ------------------------------------------------------------ */

/* Icmpv4Type::from != Unknown (misc.rs:93-119). */
static int icmpv4_known(uint8_t t) {
    static const uint8_t k[] = {0, 3, 4, 5, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18,
                                30, 40, 42, 43, 253, 254};
    for (size_t i = 0; i < sizeof k; ++i) if (k[i] == t) return 1;
    return 0;
}

/* Icmpv6Type::from != Unknown (misc.rs:164-204). */
static int icmpv6_known(uint8_t t) {
    static const uint8_t k[] = {1, 2, 3, 4, 100, 101, 128, 129, 130, 131, 132, 133, 134,
                                135, 136, 137, 138, 139, 140, 141, 142, 143, 144, 145,
                                146, 147, 148, 149, 150, 151, 152, 153, 155, 200, 201};
    for (size_t i = 0; i < sizeof k; ++i) if (k[i] == t) return 1;
    return 0;
}

/* ---- parser state (parser.rs:22-32) ------------------------------------ */

typedef struct {
    int present;
    size_t start;                   /* offset of the reader's slice in the frame */
} opt_t;

typedef struct {                    /* extensions/headers.rs:19-28 */
    opt_t h[ZP_EXT_SLOTS];          /* hop_by_hop, routing, fragment, auth, dest1, dest2 */
    size_t total_headers_len;
    uint8_t final_next_header;
} ext_t;

typedef struct {                    /* ipv6.rs:135-142 */
    slice_t bytes;
    int has_ext;
    ext_t ext;
    size_t extension_headers_len;
} ipv6_t;

typedef struct {
    const uint8_t* frame;
    opt_t ethernet, arp, ipv4, ipv6, ip_in_ip, tcp, udp, icmpv4, icmpv6;
    int ip_in_ip_v6;
    size_t eth_header_len;
    ipv6_t outer6, inner6;          /* reader payloads kept for the record */
} parser_t;

static size_t off_of(const parser_t* ps, slice_t s) { return (size_t)(s.p - ps->frame); }

/* ---- extension headers (headers.rs:51-213) ------------------------------ */

static int ext_is_empty(const ext_t* e) {                    /* :206-213 */
    for (int k = 0; k < ZP_EXT_SLOTS; ++k) if (e->h[k].present) return 0;
    return 1;
}

/* One step of the walk (headers.rs:73-86). Returns 0 and *more = 1 with the
 * next (header, bytes) to continue, *more = 0 to stop, or an error. */
static int ext_step(ext_t* e, const uint8_t* payload_start, uint8_t nh, slice_t bytes,
                    int* more, uint8_t* next_nh, slice_t* next_bytes) {
    int slot;
    size_t min_len, hl;
    int err_short, err_exceeds;
    *more = 0;
    switch (nh) {
    case 0:                                                     /* :90-113 */
        if (e->h[ZP_EXT_HBH].present) return 0;
        if (!ext_is_empty(e)) return ZP_ERR_EXT_HBH_NOT_FIRST;
        slot = ZP_EXT_HBH; min_len = 8;
        err_short = ZP_ERR_EXT_OPTIONS_TOO_SHORT; err_exceeds = ZP_ERR_EXT_OPTIONS_EXCEEDS;
        break;
    case 43:                                                    /* :117-134 */
        if (e->h[ZP_EXT_RT].present) return 0;
        slot = ZP_EXT_RT; min_len = 8;
        err_short = ZP_ERR_EXT_ROUTING_TOO_SHORT; err_exceeds = ZP_ERR_EXT_ROUTING_EXCEEDS;
        break;
    case 44:                                                    /* :138-155 */
        if (e->h[ZP_EXT_FRAG].present) return 0;
        slot = ZP_EXT_FRAG; min_len = 8;
        err_short = ZP_ERR_EXT_FRAGMENT_TOO_SHORT; err_exceeds = 0;
        break;
    case 51:                                                    /* :159-176 */
        if (e->h[ZP_EXT_AH].present) return 0;
        slot = ZP_EXT_AH; min_len = 12;
        err_short = ZP_ERR_EXT_AUTH_TOO_SHORT; err_exceeds = ZP_ERR_EXT_AUTH_EXCEEDS;
        break;
    case 60:                                                    /* :180-202 */
        if (e->h[ZP_EXT_DST2].present) return 0;
        slot = e->h[ZP_EXT_DST1].present ? ZP_EXT_DST2 : ZP_EXT_DST1; min_len = 8;
        err_short = ZP_ERR_EXT_OPTIONS_TOO_SHORT; err_exceeds = ZP_ERR_EXT_OPTIONS_EXCEEDS;
        break;
    default:
        return 0;                                               /* :84 */
    }
    if (bytes.n < min_len) return err_short;                    /* Reader::new */
    uint8_t next = bytes.p[0];                                  /* next_header() */
    if (slot == ZP_EXT_FRAG) hl = 8;                            /* fragment.rs:160-162 */
    else if (slot == ZP_EXT_AH) hl = ((size_t)bytes.p[1] + 2) * 4;   /* authentication.rs:178-181 */
    else hl = ((size_t)bytes.p[1] + 1) * 8;                     /* options.rs:127-130, routing.rs:172-175 */
    if (err_exceeds && hl > bytes.n) return err_exceeds;        /* payload()? */
    e->total_headers_len += hl;
    e->final_next_header = next;
    e->h[slot].present = 1;
    e->h[slot].start = (size_t)(bytes.p - payload_start);
    *more = 1;
    *next_nh = next;
    *next_bytes = sub(bytes, hl);
    return 0;
}

/* ExtensionHeaders::parse (headers.rs:51-69). */
static int ext_parse(slice_t bytes, uint8_t next_header, ext_t* e, int* some) {
    memset(e, 0, sizeof *e);
    const uint8_t* payload_start = bytes.p;
    uint8_t cur = next_header;
    slice_t cb = bytes;
    for (;;) {
        int more;
        uint8_t nnh;
        slice_t nb;
        int err = ext_step(e, payload_start, cur, cb, &more, &nnh, &nb);
        if (err) return err;
        if (!more) break;
        cur = nnh;
        cb = nb;
    }
    *some = !ext_is_empty(e);
    return 0;
}

/* IPv6Reader::new (ipv6.rs:147-167). */
static int ipv6_new(slice_t bytes, ipv6_t* r) {
    if (bytes.n < 40) return ZP_ERR_IPV6_TOO_SHORT;
    memset(r, 0, sizeof *r);
    r->bytes = bytes;
    int some = 0;
    int err = ext_parse(sub(bytes, 40), bytes.p[6], &r->ext, &some);
    if (err) return err;
    if (some) {
        r->has_ext = 1;
        r->extension_headers_len = r->ext.total_headers_len;
    }
    return 0;
}

/* IPv6Reader::final_next_header (ipv6.rs:219-227). */
static uint8_t ipv6_final_nh(const ipv6_t* r) {
    return r->has_ext ? r->ext.final_next_header : r->bytes.p[6];
}

/* ---- parser.rs ----------------------------------------------------------- */

static int parse_ipv4(parser_t* ps, slice_t payload, int from_ether);
static int parse_ipv6(parser_t* ps, slice_t payload, int from_ether);

/* The enclosing IP header for VerifyReader (parser.rs:306-362). */
typedef struct {
    int v6;
    slice_t ip;          /* IPv4 reader bytes / IPv6 reader bytes */
    slice_t payload;     /* IPv4 payload() / IPv6 upper_layer_payload() */
    uint8_t proto;       /* IPv4 protocol() / IPv6 final_next_header() */
} verify_t;

static int verify_checksum(const verify_t* v) {
    if (!v->v6) {                                               /* :316-333 */
        uint32_t sum = v->proto == 1 ? 0
            : zpo_pseudo_header(v->ip.p + 12, v->ip.p + 16, 4, v->proto, v->payload.n);
        if (!verify_internet_checksum(v->payload, sum)) return ZP_ERR_IPV4_L4_CHECKSUM;
        return 0;
    }
    if (v->proto == 59) return 0;                               /* :342-344 */
    uint32_t sum = zpo_pseudo_header(v->ip.p + 8, v->ip.p + 24, 16, v->proto, v->payload.n);
    if (!verify_internet_checksum(v->payload, sum)) return ZP_ERR_IPV6_L4_CHECKSUM;
    return 0;
}

/* parse_protocol (parser.rs:111-140) with the L4 ParseReader impls (:233-303). */
static int parse_protocol(parser_t* ps, uint8_t protocol, slice_t payload, const verify_t* v) {
    int err;
    switch (protocol) {
    case 6:                                                     /* :118-121, :238-250 */
        if (payload.n < 20) return ZP_ERR_TCP_TOO_SHORT;        /* tcp.rs:142-144 */
        if ((size_t)(payload.p[12] >> 4) * 4 < 20) return ZP_ERR_TCP_DATA_OFFSET;
        if (payload.p[13] == 0) return ZP_ERR_TCP_FLAGS;
        ps->tcp.present = 1; ps->tcp.start = off_of(ps, payload);
        return verify_checksum(v);
    case 17:                                                    /* :122-125, :258-266 */
        if (payload.n < 8) return ZP_ERR_UDP_TOO_SHORT;         /* udp.rs:104-106 */
        if ((size_t)be16(payload, 4) != 8 + (payload.n - 8)) return ZP_ERR_UDP_LENGTH;
        ps->udp.present = 1; ps->udp.start = off_of(ps, payload);
        return verify_checksum(v);
    case 1:                                                     /* :126-129, :274-286 */
        if (payload.n < 8) return ZP_ERR_ICMP_TOO_SHORT;        /* icmpv4.rs:93-95 */
        if (!icmpv4_known(payload.p[0])) return ZP_ERR_ICMPV4_TYPE;
        if (payload.p[1] > 15) return ZP_ERR_ICMPV4_CODE;       /* icmpv4.rs:8 */
        ps->icmpv4.present = 1; ps->icmpv4.start = off_of(ps, payload);
        return verify_checksum(v);
    case 58:                                                    /* :130-133, :294-302 */
        if (payload.n < 8) return ZP_ERR_ICMP_TOO_SHORT;        /* icmpv6.rs:90-92 */
        if (!icmpv6_known(payload.p[0])) return ZP_ERR_ICMPV6_TYPE;
        ps->icmpv6.present = 1; ps->icmpv6.start = off_of(ps, payload);
        return verify_checksum(v);
    case 4:                                                     /* :134 */
        return parse_ipv4(ps, payload, 0);
    case 41:                                                    /* :135 */
        return parse_ipv6(ps, payload, 0);
    default:                                                    /* :136 */
        (void)err;
        return 0;
    }
}

/* parse_ipv4 (parser.rs:73-88) with ParseReader for IPv4Reader (:188-212). */
static int parse_ipv4(parser_t* ps, slice_t b, int from_ether) {
    if (b.n < 20) return ZP_ERR_IPV4_TOO_SHORT;                 /* ipv4.rs:139-141 */
    if ((b.p[0] >> 4) != 4) return ZP_ERR_IPV4_VERSION;         /* :191 */
    size_t hl = (size_t)(b.p[0] & 0x0F) * 4;                    /* ipv4.rs:230-232 */
    if (hl < 20) return ZP_ERR_IPV4_IHL_TOO_SHORT;              /* :195 */
    if (b.n < hl) return ZP_ERR_IPV4_HDR_TOO_LONG;              /* :199 */
    if (b.n != (size_t)be16(b, 2)) return ZP_ERR_IPV4_TOTAL_LENGTH;  /* :203 */
    if (zpo_internet_checksum(b.p, hl, 0) != 0) return ZP_ERR_IPV4_CHECKSUM;  /* :207, ipv4.rs:262 */
    slice_t payload = sub(b, hl);                               /* ipv4.rs:250-258 */
    verify_t v = {0, b, payload, b.p[9]};
    int err = parse_protocol(ps, b.p[9], payload, &v);
    if (err) return err;
    if (from_ether) {
        ps->ipv4.present = 1; ps->ipv4.start = off_of(ps, b);
    } else {                                                    /* overwritten by outer levels */
        ps->ip_in_ip.present = 1; ps->ip_in_ip.start = off_of(ps, b); ps->ip_in_ip_v6 = 0;
    }
    return 0;
}

/* parse_ipv6 (parser.rs:92-107) with ParseReader for IPv6Reader (:222-230). */
static int parse_ipv6(parser_t* ps, slice_t b, int from_ether) {
    ipv6_t r;
    int err = ipv6_new(b, &r);
    if (err) return err;
    if ((b.p[0] >> 4) != 6) return ZP_ERR_IPV6_VERSION;         /* :225 */
    slice_t ulp = sub(b, 40 + r.extension_headers_len);         /* ipv6.rs:283-285 */
    uint8_t nh = ipv6_final_nh(&r);
    verify_t v = {1, b, ulp, nh};
    err = parse_protocol(ps, nh, ulp, &v);
    if (err) return err;
    if (from_ether) {
        ps->ipv6.present = 1; ps->ipv6.start = off_of(ps, b); ps->outer6 = r;
    } else {
        ps->ip_in_ip.present = 1; ps->ip_in_ip.start = off_of(ps, b); ps->ip_in_ip_v6 = 1;
        ps->inner6 = r;
    }
    return 0;
}

/* PacketParser::parse (parser.rs:53-69). */
static int parse(parser_t* ps, slice_t bytes) {
    memset(ps, 0, sizeof *ps);
    ps->frame = bytes.p;
    if (bytes.n < 64) return ZP_ERR_ETH_FRAME_TOO_SHORT;       /* :159-161 */
    if (bytes.n < 14) return ZP_ERR_ETH_SLICE_TOO_SHORT;       /* ethernet.rs:142 */
    size_t hl;                                                  /* ethernet.rs:155-179 */
    switch (be16(bytes, 12)) {
    case 0x8100:
        if (bytes.n < 18) return ZP_ERR_ETH_VLAN_TOO_SHORT;
        hl = 18;
        break;
    case 0x88A8:
        if (bytes.n < 22) return ZP_ERR_ETH_QINQ_TOO_SHORT;
        if (be16(bytes, 16) != 0x8100) return ZP_ERR_ETH_INVALID_QINQ;
        hl = 22;
        break;
    default:
        hl = 14;
    }
    slice_t payload = sub(bytes, hl);
    uint16_t ethertype = be16(bytes, hl - 2);                   /* ethernet.rs:209-212 */
    int err = 0;
    if (ethertype == 0x0806) {                                  /* :60, :172-180 */
        if (payload.n < 28) return ZP_ERR_ARP_TOO_SHORT;        /* arp.rs:131-133 */
        if (be16(payload, 6) > 2) return ZP_ERR_ARP_INVALID_OPER;
        ps->arp.present = 1; ps->arp.start = hl;
    } else if (ethertype == 0x0800) {
        err = parse_ipv4(ps, payload, 1);
    } else if (ethertype == 0x86DD) {
        err = parse_ipv6(ps, payload, 1);
    }
    if (err) return err;
    ps->ethernet.present = 1; ps->ethernet.start = 0;
    ps->eth_header_len = hl;
    return 0;
}

/* ---- record encoding (include/zero_packet.h) ----------------------------- */

/* The oracle's result of one frame, every field unpacked (the layout of the
 * ABI v2/v3 record). zpo_pack encodes it as the ABI's 8-B zp_record, which
 * the tests compare with the GPU's byte for byte; the field-level tests read
 * this form. final_nh / inner_final_nh: IPv6Reader::final_next_header
 * (ipv6.rs:219-227) of the outer / ip_in_ip IPv6 (in the ABI: the ext entry
 * of a chain, else the header's next-header byte). */
typedef struct zpo_record {
    uint32_t flags;
    uint8_t  err, eth_len, final_nh, inner_final_nh;
    uint32_t inner_off, l4_off;
} zpo_record;

/* The inline code of an outer chain (ZP_CHAIN_INLINE, include/zero_packet.h,
 * ABI v6) from the record and the chain's entry, or 0 when the chain does not
 * go inline: the present headers sorted by offset must come in RFC 8200 order
 * (Hop-by-Hop, Destination 1st, Routing, Fragment, Authentication,
 * Destination 2nd) with lengths their code fields hold, and the frame needs an
 * L4 reader and no ip_in_ip header. */
static uint32_t chain_code(const zpo_record* r, const zp_ext_offsets* x) {
    static const int rfc[6] = {ZP_EXT_HBH, ZP_EXT_DST1, ZP_EXT_RT, ZP_EXT_FRAG, ZP_EXT_AH,
                               ZP_EXT_DST2};
    const uint32_t l4 = ZP_F_TCP | ZP_F_UDP | ZP_F_ICMPV4 | ZP_F_ICMPV6;
    if (!x || (r->flags & (ZP_F_EXT | ZP_F_IP_IN_IP)) != ZP_F_EXT || !(r->flags & l4) ||
        r->l4_off > ZP_L4_NEAR_MAX)
        return 0;
    int seq[6], m = 0;
    for (int j = 0; j < 6; ++j)
        if (r->flags & ZP_F_EXT_SLOT(rfc[j])) seq[m++] = rfc[j];
    uint32_t code = ZP_CHAIN_INLINE >> 18, at = 0;
    for (int q = 0; q < m; ++q) {
        const int k = seq[q];
        if (x->off[k] != at) return 0;                      /* not in RFC order */
        const uint32_t end = q + 1 < m ? x->off[seq[q + 1]] : x->len;
        if (end <= at) return 0;
        const uint32_t hl = end - at;
        if (k == ZP_EXT_FRAG) {
            if (hl != 8) return 0;
        } else if (k == ZP_EXT_AH) {
            if (hl % 4 || hl / 4 - 2 > 3) return 0;
            code |= (hl / 4 - 2) << 8;
        } else {
            const uint32_t c = hl / 8 - 1, cmax = (k == ZP_EXT_HBH || k == ZP_EXT_RT) ? 7u : 3u;
            if (hl % 8 || c > cmax) return 0;
            code |= c << (k == ZP_EXT_HBH ? 0 : k == ZP_EXT_RT ? 5 : k == ZP_EXT_DST1 ? 3 : 10);
        }
        at = end;
    }
    return code;
}

/* zp_record (include/zero_packet.h): flags | Ethernet code << 24 | err << 26,
 * l4_off | inner_off << 18, or the outer chain's inline code in bits 18-31
 * (ABI v6; outer = the n outer-chain entries, NULL: no inline chains); an
 * l4_off past ZP_L4_NEAR_MAX in the far-L4 form (code 3, offs = l4_off; ABI
 * v5). */
void zpo_pack(const zpo_record* full, const zp_ext_offsets* outer, uint64_t n, zp_record* out) {
    for (uint64_t i = 0; i < n; ++i) {
        const zpo_record* r = &full[i];
        if (r->err) {
            out[i].flags = (uint32_t)r->err << 26;
            out[i].offs = 0;
            continue;
        }
        if (r->l4_off > ZP_L4_NEAR_MAX) {
            out[i].flags = r->flags | ZP_ETH_CODE_FAR << 24;
            out[i].offs = r->l4_off;
            continue;
        }
        const uint32_t code = chain_code(r, outer ? &outer[i] : NULL);
        out[i].flags = r->flags | ((uint32_t)(r->eth_len - 14) / 4u) << 24;
        out[i].offs = r->l4_off | (code ? code : r->inner_off) << 18;
    }
}

/* One Option<ExtensionHeaders> (headers.rs:19-28) -> slot bits + a
 * zp_ext_offsets entry (len = extension_headers_len, ipv6.rs:141). */
static void ext_to_record(const ipv6_t* r, uint32_t shift, uint32_t* flags, zp_ext_offsets* x) {
    x->len = (uint16_t)r->extension_headers_len;
    x->final_nh = ipv6_final_nh(r);                 /* headers.rs:26 */
    for (int k = 0; k < ZP_EXT_SLOTS; ++k) {
        if (r->ext.h[k].present) {
            *flags |= 1u << (shift + k);
            x->off[k] = (uint16_t)r->ext.h[k].start;
        }
    }
}

/* One frame: the record, and (xo / xi non-NULL) the outer and ip_in_ip
 * extension chains; entries without a chain are zero. */
int zpo_parse(const uint8_t* frame, size_t len, zpo_record* rec, zp_ext_offsets* xo,
              zp_ext_offsets* xi) {
    parser_t ps;
    slice_t s = {frame, len};
    int err = parse(&ps, s);
    zp_ext_offsets to, ti;
    memset(rec, 0, sizeof *rec);
    memset(&to, 0, sizeof to);
    memset(&ti, 0, sizeof ti);
    if (xo) *xo = to;
    if (xi) *xi = ti;
    if (err) { rec->err = (uint8_t)err; return err; }
    uint32_t f = 0;
    if (ps.ethernet.present) f |= ZP_F_ETHERNET;
    if (ps.arp.present) f |= ZP_F_ARP;
    if (ps.ipv4.present) f |= ZP_F_IPV4;
    if (ps.ipv6.present) f |= ZP_F_IPV6;
    if (ps.tcp.present) { f |= ZP_F_TCP; rec->l4_off = (uint32_t)ps.tcp.start; }
    if (ps.udp.present) { f |= ZP_F_UDP; rec->l4_off = (uint32_t)ps.udp.start; }
    if (ps.icmpv4.present) { f |= ZP_F_ICMPV4; rec->l4_off = (uint32_t)ps.icmpv4.start; }
    if (ps.icmpv6.present) { f |= ZP_F_ICMPV6; rec->l4_off = (uint32_t)ps.icmpv6.start; }
    rec->eth_len = (uint8_t)ps.eth_header_len;
    if (ps.ipv6.present) {
        rec->final_nh = ipv6_final_nh(&ps.outer6);
        if (ps.outer6.has_ext) {
            f |= ZP_F_EXT;
            ext_to_record(&ps.outer6, 12, &f, &to);
            if (xo) *xo = to;
        }
    }
    if (ps.ip_in_ip.present) {
        f |= ZP_F_IP_IN_IP;
        rec->inner_off = (uint32_t)ps.ip_in_ip.start;
        if (ps.ip_in_ip_v6) {
            f |= ZP_F_IP_IN_IP_V6;
            rec->inner_final_nh = ipv6_final_nh(&ps.inner6);
            if (ps.inner6.has_ext) {
                f |= ZP_F_INNER_EXT;
                ext_to_record(&ps.inner6, 18, &f, &ti);
                if (xi) *xi = ti;
            }
        }
    }
    rec->flags = f;
    return 0;
}

/* ---- standalone reader constructors (README.md:110-115) ------------------ */

/* XReader::new(bytes) of reader `kind` (zp_reader_kind order). Returns 0 or
 * the zp_err code; *hl = Ethernet header_len, and for IPv6 *flags = ZP_F_EXT
 * + slot bits, *final_nh and *x the chain (zeros where absent). */
int zpo_reader_new(int kind, const uint8_t* b, size_t n, uint32_t* hl, uint32_t* flags,
                   uint8_t* final_nh, zp_ext_offsets* x) {
    slice_t s = {b, n};
    *hl = 0; *flags = 0; *final_nh = 0;
    memset(x, 0, sizeof *x);
    switch (kind) {
    case 0:                                                     /* ethernet.rs:141-179 */
        if (n < 14) return ZP_ERR_ETH_SLICE_TOO_SHORT;          /* :142-144 */
        switch (be16(s, 12)) {
        case 0x8100:
            if (n < 18) return ZP_ERR_ETH_VLAN_TOO_SHORT;       /* :159-161 */
            *hl = 18;
            return 0;
        case 0x88A8:
            if (n < 22) return ZP_ERR_ETH_QINQ_TOO_SHORT;       /* :166-168 */
            if (be16(s, 16) != 0x8100) return ZP_ERR_ETH_INVALID_QINQ;   /* :171-173 */
            *hl = 22;
            return 0;
        default:
            *hl = 14;
            return 0;
        }
    case 1: return n < 28 ? ZP_ERR_ARP_TOO_SHORT : 0;           /* arp.rs:130-134 */
    case 2: return n < 20 ? ZP_ERR_IPV4_TOO_SHORT : 0;          /* ipv4.rs:138-142 */
    case 3: {                                                   /* ipv6.rs:147-167 */
        ipv6_t r;
        int err = ipv6_new(s, &r);
        if (err) return err;
        *final_nh = ipv6_final_nh(&r);
        if (r.has_ext) {
            *flags = ZP_F_EXT;
            ext_to_record(&r, 12, flags, x);
        }
        return 0;
    }
    case 4: return n < 8 ? ZP_ERR_EXT_OPTIONS_TOO_SHORT : 0;    /* options.rs:83-87 */
    case 5: return n < 8 ? ZP_ERR_EXT_ROUTING_TOO_SHORT : 0;    /* routing.rs:107-111 */
    case 6: return n < 8 ? ZP_ERR_EXT_FRAGMENT_TOO_SHORT : 0;   /* fragment.rs:97-101 */
    case 7: return n < 12 ? ZP_ERR_EXT_AUTH_TOO_SHORT : 0;      /* authentication.rs:105-109 */
    case 8: return n < 20 ? ZP_ERR_TCP_TOO_SHORT : 0;           /* tcp.rs:141-145 */
    case 9: return n < 8 ? ZP_ERR_UDP_TOO_SHORT : 0;            /* udp.rs:103-107 */
    case 10: return n < 8 ? ZP_ERR_ICMP_TOO_SHORT : 0;          /* icmpv4.rs:92-96 */
    case 11: return n < 8 ? ZP_ERR_ICMP_TOO_SHORT : 0;          /* icmpv6.rs:89-93 */
    }
    return -1;
}

/* ---- batch driver (CPU baseline) ----------------------------------------- */

typedef struct {
    const uint8_t* arena;
    const uint64_t* offs;
    const uint32_t* lens;
    zpo_record* recs;
    zp_ext_offsets* ext;        /* 2n entries or NULL */
    uint64_t n, lo, hi;
} job_t;

static void* worker(void* a) {
    job_t* j = (job_t*)a;
    for (uint64_t i = j->lo; i < j->hi; ++i)
        zpo_parse(j->arena + j->offs[i], j->lens[i], &j->recs[i], j->ext ? &j->ext[i] : 0,
                  j->ext ? &j->ext[j->n + i] : 0);
    return 0;
}

/* Parses n frames with `nthreads` threads over contiguous shards
 * (nthreads <= 0: all online cores); ext: NULL or 2n entries laid out as
 * zp_parse_batch_device's. Returns the thread count used. */
int zpo_parse_batch(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                    uint64_t n, zpo_record* recs, zp_ext_offsets* ext, int nthreads) {
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads > 256) nthreads = 256;
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    int started[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (job_t){arena, offs, lens, recs, ext, n, n * t / nthreads, n * (t + 1) / nthreads};
        started[t] = 0;
        if (nthreads == 1) { worker(&jobs[t]); continue; }
        if (pthread_create(&th[t], 0, worker, &jobs[t]) == 0) started[t] = 1;
        else worker(&jobs[t]);
    }
    for (int t = 0; t < nthreads; ++t) if (started[t]) pthread_join(th[t], 0);
    return nthreads;
}

/* ---- column views -------------------------------- */
/* The reader getters restated over the frame bytes at the record's offsets:
 * EthernetReader (ethernet.rs:195-244), ArpReader::oper (arp.rs:174-177),
 * IPv4Reader (ipv4.rs:148-227), IPv6Reader (ipv6.rs:173-256), TcpReader
 * (tcp.rs:151-243), UdpReader (udp.rs:113-154), Icmpv4/6Reader
 * (icmpv4.rs:102-135, icmpv6.rs:99-132). The record says which readers the
 * parser holds (parser.rs:22-32); include/zero_packet.h defines each column. */

static const int col_width[ZP_COL_COUNT] = {
    6, 6, 2, 2, 2, 2, 1, 16, 16, 1, 1, 1, 4, 2, 1, 16, 16, 1, 1, 2, 2, 4, 4, 1, 2, 1, 1, 2, 4};

static void put(void* const* cols, int c, uint64_t i, const void* v) {
    if (cols[c]) memcpy((uint8_t*)cols[c] + i * (uint64_t)col_width[c], v, (size_t)col_width[c]);
}
static void put8(void* const* cols, int c, uint64_t i, uint8_t v) { put(cols, c, i, &v); }
static void put16(void* const* cols, int c, uint64_t i, uint16_t v) { put(cols, c, i, &v); }
static void put32(void* const* cols, int c, uint64_t i, uint32_t v) { put(cols, c, i, &v); }
static uint32_t be32(slice_t s, size_t i) {
    return ((uint32_t)s.p[i] << 24) | ((uint32_t)s.p[i + 1] << 16) | ((uint32_t)s.p[i + 2] << 8) |
           s.p[i + 3];
}

/* One IP reader (outer: c0 = ZP_COL_IP_VERSION, inner: ZP_COL_INNER_VERSION). */
static void ip_columns(void* const* cols, uint64_t i, slice_t ip, int v6, uint8_t final_nh,
                       int inner) {
    uint8_t src[16] = {0}, dst[16] = {0};
    const int cv = inner ? ZP_COL_INNER_VERSION : ZP_COL_IP_VERSION;
    const int cs = inner ? ZP_COL_INNER_SRC_ADDR : ZP_COL_SRC_ADDR;
    const int cd = inner ? ZP_COL_INNER_DEST_ADDR : ZP_COL_DEST_ADDR;
    const int cp = inner ? ZP_COL_INNER_PROTOCOL : ZP_COL_PROTOCOL;
    if (!v6) {
        put8(cols, cv, i, (uint8_t)(ip.p[0] >> 4));               /* ipv4.rs:148-151 */
        memcpy(src, ip.p + 12, 4);                                 /* ipv4.rs:210-213 */
        memcpy(dst, ip.p + 16, 4);                                 /* ipv4.rs:216-219 */
        put8(cols, cp, i, ip.p[9]);                                /* ipv4.rs:204-207 */
    } else {
        put8(cols, cv, i, (uint8_t)(ip.p[0] >> 4));               /* ipv6.rs:173-176 */
        memcpy(src, ip.p + 8, 16);                                 /* ipv6.rs:245-248 */
        memcpy(dst, ip.p + 24, 16);                                /* ipv6.rs:253-256 */
        put8(cols, cp, i, final_nh);                               /* ipv6.rs:219-227 */
    }
    put(cols, cs, i, src);
    put(cols, cd, i, dst);
    if (inner) return;
    if (!v6) {
        put8(cols, ZP_COL_TTL, i, ip.p[8]);                        /* ipv4.rs:198-201 */
        put8(cols, ZP_COL_TOS, i, ip.p[1]);                        /* dscp<<2|ecn :160-169 */
        put32(cols, ZP_COL_IP_ID, i, be16(ip, 4));                 /* ipv4.rs:180-183 */
        put16(cols, ZP_COL_IP_LEN, i, be16(ip, 2));                /* ipv4.rs:174-177 */
    } else {
        put8(cols, ZP_COL_TTL, i, ip.p[7]);                        /* ipv6.rs:237-240 */
        put8(cols, ZP_COL_TOS, i,                                  /* ipv6.rs:181-186 */
             (uint8_t)(((ip.p[0] & 0x0F) << 4) | (ip.p[1] >> 4)));
        put32(cols, ZP_COL_IP_ID, i,                               /* ipv6.rs:189-196 */
              ((uint32_t)(ip.p[1] & 0x0F) << 16) | ((uint32_t)ip.p[2] << 8) | ip.p[3]);
        put16(cols, ZP_COL_IP_LEN, i, be16(ip, 4));                /* ipv6.rs:199-202 */
    }
}

int zpo_columns(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                const zpo_record* recs, uint64_t n, void* const* cols) {
    for (int c = 0; c < ZP_COL_COUNT; ++c)
        if (cols[c]) memset(cols[c], 0, n * (uint64_t)col_width[c]);
    for (uint64_t i = 0; i < n; ++i) {
        const zpo_record* r = &recs[i];
        if (r->err || !(r->flags & ZP_F_ETHERNET)) continue;
        slice_t fr = {arena + offs[i], lens[i]};
        const uint32_t hl = r->eth_len;
        put(cols, ZP_COL_DEST_MAC, i, fr.p);                       /* ethernet.rs:195-198 */
        put(cols, ZP_COL_SRC_MAC, i, fr.p + 6);                    /* ethernet.rs:201-204 */
        put16(cols, ZP_COL_ETHERTYPE, i, be16(fr, hl - 2));        /* ethernet.rs:209-212 */
        if (be16(fr, 12) == 0x8100) {                              /* vlan_tag :218-229 */
            put16(cols, ZP_COL_VLAN_TCI, i, be16(fr, 14));
        } else if (be16(fr, 12) == 0x88A8) {                       /* double_vlan_tag :232-244 */
            put16(cols, ZP_COL_VLAN_TCI, i, be16(fr, 14));
            put16(cols, ZP_COL_VLAN_INNER_TCI, i, be16(fr, 18));
        }
        if (r->flags & ZP_F_ARP) put16(cols, ZP_COL_ARP_OPER, i, be16(sub(fr, hl), 6));
        if (r->flags & (ZP_F_IPV4 | ZP_F_IPV6))
            ip_columns(cols, i, sub(fr, hl), (r->flags & ZP_F_IPV6) != 0, r->final_nh, 0);
        if (r->flags & ZP_F_IP_IN_IP)
            ip_columns(cols, i, sub(fr, r->inner_off), (r->flags & ZP_F_IP_IN_IP_V6) != 0,
                       r->inner_final_nh, 1);
        const uint32_t l4f = r->flags & (ZP_F_TCP | ZP_F_UDP | ZP_F_ICMPV4 | ZP_F_ICMPV6);
        if (!l4f) continue;
        slice_t l4 = sub(fr, r->l4_off);
        uint32_t hlen;
        if (l4f == ZP_F_TCP) {
            put8(cols, ZP_COL_L4_PROTO, i, 6);
            put16(cols, ZP_COL_SRC_PORT, i, be16(l4, 0));          /* tcp.rs:151-154 */
            put16(cols, ZP_COL_DEST_PORT, i, be16(l4, 2));         /* tcp.rs:157-160 */
            put32(cols, ZP_COL_TCP_SEQ, i, be32(l4, 4));           /* tcp.rs:163-170 */
            put32(cols, ZP_COL_TCP_ACK, i, be32(l4, 8));           /* tcp.rs:172-179 */
            put8(cols, ZP_COL_TCP_FLAGS, i, l4.p[13]);             /* tcp.rs:193-196 */
            put16(cols, ZP_COL_TCP_WINDOW, i, be16(l4, 14));       /* tcp.rs:199-202 */
            put16(cols, ZP_COL_L4_CHECKSUM, i, be16(l4, 16));      /* tcp.rs:205-208 */
            hlen = (uint32_t)(l4.p[12] >> 4) * 4;                  /* tcp.rs:217-220 */
        } else if (l4f == ZP_F_UDP) {
            put8(cols, ZP_COL_L4_PROTO, i, 17);
            put16(cols, ZP_COL_SRC_PORT, i, be16(l4, 0));          /* udp.rs:113-116 */
            put16(cols, ZP_COL_DEST_PORT, i, be16(l4, 2));         /* udp.rs:119-122 */
            put16(cols, ZP_COL_L4_CHECKSUM, i, be16(l4, 6));       /* udp.rs:125-128 */
            hlen = 8;                                              /* udp.rs:139-142 */
        } else {
            put8(cols, ZP_COL_L4_PROTO, i, l4f == ZP_F_ICMPV4 ? 1 : 58);
            put8(cols, ZP_COL_ICMP_TYPE, i, l4.p[0]);              /* icmpv4.rs:102-105 */
            put8(cols, ZP_COL_ICMP_CODE, i, l4.p[1]);              /* icmpv4.rs:108-111 */
            put16(cols, ZP_COL_L4_CHECKSUM, i, be16(l4, 2));       /* icmpv4.rs:114-117 */
            hlen = 8;                                              /* icmpv4.rs:120-123 */
        }
        if (hlen <= l4.n)                                          /* tcp.rs:235-243 */
            put32(cols, ZP_COL_PAYLOAD_OFF, i, r->l4_off + hlen);
    }
    return 0;
}

/* ---- PacketBuilder restatement -------------------- */
/* builder.rs:55-909 with the writers it calls (ethernet.rs:19-129,
 * arp.rs:7-119, ipv4.rs:8-127, ipv6.rs:8-133, options.rs / routing.rs /
 * fragment.rs / authentication.rs writers, tcp.rs:7-130, udp.rs:7-92,
 * icmpv4.rs:10-81, icmpv6.rs:7-78). One chain of ops over one buffer; the
 * first Err stops the chain with its partial writes left in the buffer. */

enum { ST_RAW, ST_ETH, ST_ARP, ST_V4, ST_V6, ST_HBH, ST_D1, ST_RT, ST_FR, ST_AH, ST_D2,
       ST_V4E, ST_V6E, ST_L4 };

/* builder.rs:817-909: the state after `kind` from `st`, or -1. */
static int next_state(int st, int kind) {
    const int l4v4 = kind == ZP_B_TCP || kind == ZP_B_UDP || kind == ZP_B_ICMPV4;
    const int l4v6 = kind == ZP_B_TCP || kind == ZP_B_UDP || kind == ZP_B_ICMPV6;
    switch (st) {
    case ST_RAW:
        return (kind == ZP_B_ETHERNET || kind == ZP_B_ETHERNET_VLAN ||
                kind == ZP_B_ETHERNET_QINQ) ? ST_ETH : -1;
    case ST_ETH:
        return kind == ZP_B_ARP ? ST_ARP : kind == ZP_B_IPV4 ? ST_V4 : kind == ZP_B_IPV6 ? ST_V6 : -1;
    case ST_V4:
        if (l4v4) return ST_L4;
        return kind == ZP_B_IPV4 ? ST_V4E : kind == ZP_B_IPV6 ? ST_V6E : -1;
    case ST_V4E: return l4v4 ? ST_L4 : -1;
    case ST_V6E: return l4v6 ? ST_L4 : -1;
    case ST_V6: case ST_HBH: case ST_D1: case ST_RT: case ST_FR: case ST_AH: case ST_D2:
        if (l4v6) return ST_L4;
        if (kind == ZP_B_IPV4) return ST_V4E;
        if (kind == ZP_B_IPV6) return ST_V6E;
        if (kind == ZP_B_HOP_BY_HOP) return st == ST_V6 ? ST_HBH : -1;
        if (kind == ZP_B_DEST_OPTS1) return (st == ST_V6 || st == ST_HBH) ? ST_D1 : -1;
        if (kind == ZP_B_ROUTING) return (st == ST_V6 || st == ST_HBH || st == ST_D1) ? ST_RT : -1;
        if (kind == ZP_B_FRAGMENT) return (st == ST_V6 || st == ST_HBH || st == ST_RT) ? ST_FR : -1;
        if (kind == ZP_B_AUTH)
            return (st == ST_V6 || st == ST_HBH || st == ST_RT || st == ST_FR) ? ST_AH : -1;
        if (kind == ZP_B_DEST_OPTS2) return st != ST_D1 && st != ST_D2 ? ST_D2 : -1;
        return -1;
    default:
        return -1;   /* ARP and L4 states are terminal */
    }
}

static void wr16(uint8_t* b, size_t i, uint16_t v) { b[i] = (uint8_t)(v >> 8); b[i + 1] = (uint8_t)v; }
static void wr32(uint8_t* b, size_t i, uint32_t v) {
    b[i] = (uint8_t)(v >> 24); b[i + 1] = (uint8_t)(v >> 16); b[i + 2] = (uint8_t)(v >> 8); b[i + 3] = (uint8_t)v;
}

/* internet_checksum over s into bytes [at, at+2) (the writers' set_checksum). */
static void put_csum(uint8_t* s, size_t n, size_t at, uint32_t acc) {
    s[at] = 0;
    s[at + 1] = 0;
    const uint16_t c = zpo_internet_checksum(s, n, acc);
    s[at] = (uint8_t)(c >> 8);
    s[at + 1] = (uint8_t)(c & 0xFF);
}

int zpo_build(uint8_t* buf, size_t n, const zp_build_op* ops, uint32_t nops,
              const uint8_t* data, zp_build_result* res) {
    memset(res, 0, sizeof *res);
    int st = ST_RAW;
    for (uint32_t k = 0; k < nops; ++k) {                 /* typestate: compile-time in Rust */
        st = next_state(st, ops[k].kind);
        if (st < 0) { res->err = ZP_BERR_TRANSITION; return ZP_BERR_TRANSITION; }
    }
    st = ST_RAW;
    size_t hl = 0;
    for (uint32_t k = 0; k < nops; ++k) {
        const zp_build_op* o = &ops[k];
        const int prev = st;
        st = next_state(st, o->kind);
        const int has_data = o->data_len != ZP_BUILD_NO_DATA;
        const uint8_t* d = data + o->data_off;
        const size_t dl = has_data ? o->data_len : 0;
        uint8_t* s = buf + hl;                           /* &mut self.bytes[self.header_len..] */
        const size_t sl = n - hl;
        int e = 0;
        switch (o->kind) {
        case ZP_B_ETHERNET: case ZP_B_ETHERNET_VLAN: case ZP_B_ETHERNET_QINQ: {
            if (n < 14) { e = ZP_BERR_ETH_SLICE; break; }                 /* ethernet.rs:29-31 */
            memcpy(buf + 6, o->src, 6);                                    /* set_src_mac :56-63 */
            memcpy(buf, o->dst, 6);                                        /* set_dest_mac :45-52 */
            size_t h = 14;
            if (o->kind == ZP_B_ETHERNET_VLAN) {                           /* set_vlan_tag :83-96 */
                if (n < h + 4) { e = ZP_BERR_ETH_VLAN; break; }
                wr16(buf, 12, 0x8100); wr16(buf, 14, o->h[1]);
                h += 4;
            } else if (o->kind == ZP_B_ETHERNET_QINQ) {                    /* :104-128 */
                if (n < h + 8) { e = ZP_BERR_ETH_QINQ; break; }
                wr16(buf, 12, 0x88A8); wr16(buf, 14, o->h[1]);
                wr16(buf, 16, 0x8100); wr16(buf, 18, o->h[2]);
                h += 8;
            }
            wr16(buf, 12 + (h - 14), o->h[0]);                             /* set_ethertype :70-74 */
            hl = h;                                                        /* builder.rs:124,155,186 */
            break;
        }
        case ZP_B_ARP:                                                     /* builder.rs:203-236 */
            if (n < hl) { e = ZP_BERR_ARP_DATA; break; }
            if (sl < 28) { e = ZP_BERR_ARP_SLICE; break; }
            wr16(s, 0, o->h[0]); wr16(s, 2, o->h[1]); s[4] = o->b[0]; s[5] = o->b[1];
            wr16(s, 6, o->h[2]);
            memcpy(s + 8, o->src, 6); memcpy(s + 14, o->src + 6, 4);
            memcpy(s + 18, o->dst, 6); memcpy(s + 24, o->dst + 6, 4);
            hl += 28;
            break;
        case ZP_B_IPV4: {                                                  /* builder.rs:248-292 */
            if (n < hl) { e = ZP_BERR_IPV4_DATA; break; }
            if (sl < 20) { e = ZP_BERR_IPV4_SLICE; break; }               /* ipv4.rs:17-19 */
            s[0] = (uint8_t)((s[0] & 0x0F) | (uint8_t)(o->b[0] << 4));    /* ipv4.rs:35-38 */
            s[0] = (uint8_t)((s[0] & 0xF0) | (o->b[1] & 0x0F));
            s[1] = (uint8_t)((s[1] & 0x03) | (uint8_t)(o->b[2] << 2));
            s[1] = (uint8_t)((s[1] & 0xFC) | (o->b[3] & 0x03));
            wr16(s, 2, o->h[0]);
            wr16(s, 4, o->h[1]);
            s[6] = (uint8_t)((s[6] & 0x1F) | ((uint8_t)(o->b[4] << 5) & 0xE0));
            s[6] = (uint8_t)((s[6] & 0xE0) | ((o->h[2] >> 8) & 0x1F));
            s[7] = (uint8_t)(o->h[2] & 0xFF);
            s[8] = o->b[5];
            s[9] = o->b[6];
            memcpy(s + 12, o->src, 4);
            memcpy(s + 16, o->dst, 4);
            const size_t ihl = (size_t)(s[0] & 0x0F) * 4;                  /* ipv4.rs:26-28 */
            s[10] = 0; s[11] = 0;                                          /* set_checksum :119-126 */
            if (ihl > sl) { e = ZP_BERR_PANIC; break; }                    /* &bytes[..header_len] */
            put_csum(s, ihl, 10, 0);
            hl += ihl;
            break;
        }
        case ZP_B_IPV6:                                                    /* builder.rs:300-335 */
            if (n < hl) { e = ZP_BERR_IPV6_DATA; break; }
            if (sl < 40) { e = ZP_BERR_IPV6_SLICE; break; }
            s[0] = (uint8_t)((s[0] & 0x0F) | (uint8_t)(o->b[0] << 4));    /* ipv6.rs:33-36 */
            s[0] = (uint8_t)((s[0] & 0xF0) | (o->b[1] >> 4));             /* :40-44 */
            s[1] = (uint8_t)((s[1] & 0x0F) | (uint8_t)(o->b[1] << 4));
            s[1] = (uint8_t)((s[1] & 0xF0) | (uint8_t)(o->w[0] >> 16));   /* :48-52 (unmasked) */
            s[2] = (uint8_t)(o->w[0] >> 8);
            s[3] = (uint8_t)o->w[0];
            wr16(s, 4, o->h[0]);
            s[6] = o->b[2];
            s[7] = o->b[3];
            memcpy(s + 8, o->src, 16);
            memcpy(s + 24, o->dst, 16);
            hl += 40;
            break;
        case ZP_B_HOP_BY_HOP: case ZP_B_DEST_OPTS1: case ZP_B_DEST_OPTS2: { /* builder.rs:611-806 */
            if (n < hl) { e = o->kind == ZP_B_HOP_BY_HOP ? ZP_BERR_HBH_DATA : ZP_BERR_DEST_DATA; break; }
            if (sl < 8) { e = ZP_BERR_OPTIONS_SLICE; break; }             /* options.rs:17-19 */
            s[0] = o->b[0];
            s[1] = o->b[1];
            if (dl < 6) { e = ZP_BERR_OPTIONS_MIN; break; }               /* options.rs:53-68 */
            if ((size_t)s[1] * 8 != dl) { e = ZP_BERR_OPTIONS_MATCH; break; }
            if (2 + dl > sl) { e = ZP_BERR_OPTIONS_EXCEED; break; }
            memcpy(s + 2, d, dl);
            hl += ((size_t)s[1] + 1) * 8;
            break;
        }
        case ZP_B_ROUTING:                                                 /* builder.rs:675-704 */
            if (n < hl) { e = ZP_BERR_ROUTING_DATA; break; }
            if (sl < 8) { e = ZP_BERR_ROUTING_SLICE; break; }
            s[0] = o->b[0]; s[1] = o->b[1]; s[2] = o->b[2]; s[3] = o->b[3];
            if (dl < 4) { e = ZP_BERR_ROUTING_MIN; break; }               /* routing.rs:75-94 */
            if ((size_t)s[1] * 8 != dl) { e = ZP_BERR_ROUTING_MATCH; break; }
            if (8 + dl > sl) { e = ZP_BERR_ROUTING_EXCEED; break; }
            memcpy(s + 8, d, dl);
            hl += ((size_t)s[1] + 1) * 8;
            break;
        case ZP_B_FRAGMENT: {                                              /* builder.rs:711-740 */
            if (n < hl) { e = ZP_BERR_ROUTING_DATA; break; }              /* (its message) */
            if (sl < 8) { e = ZP_BERR_PANIC; break; }                     /* fragment.rs:15-17 panic! */
            s[0] = o->b[0];
            s[1] = 0;
            const uint16_t v = o->h[0] & 0x1FFF;                          /* fragment.rs:52-57 */
            s[2] = (uint8_t)(v >> 5);
            s[3] = (uint8_t)((s[3] & 0xE0) | (v & 0x1F));
            s[3] = (uint8_t)(s[3] & 0x9F);                                /* set_res(0) */
            if (o->b[1]) s[3] |= 0x80; else s[3] &= 0x7F;                 /* set_m_flag */
            wr32(s, 4, o->w[0]);
            hl += 8;
            break;
        }
        case ZP_B_AUTH:                                                    /* builder.rs:747-778 */
            if (n < hl) { e = ZP_BERR_AUTH_DATA; break; }
            if (sl < 12) { e = ZP_BERR_AUTH_SLICE; break; }
            s[0] = o->b[0]; s[1] = o->b[1]; s[2] = 0; s[3] = 0;
            wr32(s, 4, o->w[0]);
            wr32(s, 8, o->w[1]);
            if (12 + dl > sl) { e = ZP_BERR_AUTH_EXCEED; break; }         /* authentication.rs:84-92 */
            memcpy(s + 12, d, dl);
            hl += ((size_t)s[1] + 2) * 4;
            break;
        case ZP_B_TCP: case ZP_B_UDP: case ZP_B_ICMPV4: case ZP_B_ICMPV6: {
            const int v4 = prev == ST_V4 || prev == ST_V4E;               /* &[u8; 4] states */
            if (n < hl) {
                e = o->kind == ZP_B_TCP ? ZP_BERR_TCP_DATA : o->kind == ZP_B_UDP ? ZP_BERR_UDP_DATA
                  : o->kind == ZP_B_ICMPV4 ? ZP_BERR_ICMPV4_DATA : ZP_BERR_ICMPV6_DATA;
                break;
            }
            size_t start;
            if (o->kind == ZP_B_TCP) {                                     /* builder.rs:438-485 */
                if (sl < 20) { e = ZP_BERR_TCP_SLICE; break; }
                wr16(s, 0, o->h[0]); wr16(s, 2, o->h[1]);
                wr32(s, 4, o->w[0]); wr32(s, 8, o->w[1]);
                s[12] = (uint8_t)((uint8_t)(o->b[0] << 4) | (s[12] & 0x0F));
                s[12] = (uint8_t)((s[12] & 0xF0) | (o->b[1] & 0x0F));
                s[13] = o->b[2];
                wr16(s, 14, o->h[2]);
                wr16(s, 18, o->h[3]);
                start = (size_t)(s[12] >> 4) * 4;
            } else if (o->kind == ZP_B_UDP) {                              /* builder.rs:492-527 */
                if (sl < 8) { e = ZP_BERR_UDP_SLICE; break; }
                wr16(s, 0, o->h[0]); wr16(s, 2, o->h[1]); wr16(s, 4, o->h[2]);
                start = 8;
            } else {                                                       /* builder.rs:534-604 */
                if (sl < 8) { e = ZP_BERR_ICMP_SLICE; break; }
                s[0] = o->b[0]; s[1] = o->b[1];
                start = 8;
            }
            if (has_data) {                                                /* set_payload */
                if (start > sl) { e = ZP_BERR_PANIC; break; }              /* tcp.rs:109-114: wrap, then slice panic */
                if (sl - start < dl) {
                    e = o->kind == ZP_B_ICMPV4 ? ZP_BERR_ICMPV4_PAYLOAD
                      : o->kind == ZP_B_ICMPV6 ? ZP_BERR_ICMPV6_PAYLOAD : ZP_BERR_TCP_PAYLOAD;
                    break;
                }
                memcpy(s + start, d, dl);
            }
            uint32_t acc = 0;
            const uint8_t proto = o->kind == ZP_B_TCP ? 6 : o->kind == ZP_B_UDP ? 17 : 58;
            if (o->kind != ZP_B_ICMPV4)                                    /* checksum.rs:66-69 */
                acc = zpo_pseudo_header(o->src, o->dst, v4 ? 4 : 16, proto, sl);
            const size_t at = o->kind == ZP_B_TCP ? 16 : o->kind == ZP_B_UDP ? 6 : 2;
            put_csum(s, sl, at, acc);
            hl += o->kind == ZP_B_TCP ? start : 8;
            break;
        }
        default:
            e = ZP_BERR_TRANSITION;
        }
        if (e) {
            res->err = (uint8_t)e;
            res->header_len = (uint32_t)hl;
            res->ops_done = (uint8_t)(k > 255 ? 255 : k);
            return e;
        }
        res->ops_done = (uint8_t)(k + 1 > 255 ? 255 : k + 1);
    }
    res->header_len = (uint32_t)hl;
    return 0;
}

int zpo_build_batch(uint8_t* arena, const uint64_t* offs, const uint32_t* lens, uint64_t n,
                    const zp_build_op* ops, const uint32_t* op_start, const uint8_t* data,
                    zp_build_result* res) {
    for (uint64_t i = 0; i < n; ++i)
        zpo_build(arena + offs[i], lens[i], ops + op_start[i], op_start[i + 1] - op_start[i],
                  data, &res[i]);
    return 0;
}
