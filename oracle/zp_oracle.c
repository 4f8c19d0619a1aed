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

static void ext_to_record(const ipv6_t* r, uint32_t shift, uint32_t* flags, uint16_t off[6]) {
    for (int k = 0; k < ZP_EXT_SLOTS; ++k) {
        if (r->ext.h[k].present) {
            *flags |= 1u << (shift + k);
            off[k] = (uint16_t)r->ext.h[k].start;
        }
    }
}

int zpo_parse(const uint8_t* frame, size_t len, zp_record* rec, zp_ext_offsets* inner) {
    parser_t ps;
    slice_t s = {frame, len};
    int err = parse(&ps, s);
    memset(rec, 0, sizeof *rec);
    if (inner) memset(inner, 0, sizeof *inner);
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
            rec->ext_len = (uint16_t)ps.outer6.extension_headers_len;
            ext_to_record(&ps.outer6, 12, &f, rec->ext_off);
        }
    }
    if (ps.ip_in_ip.present) {
        f |= ZP_F_IP_IN_IP;
        rec->inner_off = (uint32_t)ps.ip_in_ip.start;
        if (ps.ip_in_ip_v6) {
            f |= ZP_F_IP_IN_IP_V6;
            rec->inner_final_nh = ipv6_final_nh(&ps.inner6);
            if (ps.inner6.has_ext) {
                zp_ext_offsets tmp;
                memset(&tmp, 0, sizeof tmp);
                f |= ZP_F_INNER_EXT;
                rec->inner_ext_len = (uint16_t)ps.inner6.extension_headers_len;
                ext_to_record(&ps.inner6, 18, &f, tmp.off);
                if (inner) *inner = tmp;
            }
        }
    }
    rec->flags = f;
    return 0;
}

/* ---- batch driver (CPU baseline) ----------------------------------------- */

typedef struct {
    const uint8_t* arena;
    const uint64_t* offs;
    const uint32_t* lens;
    zp_record* recs;
    zp_ext_offsets* inner;
    uint64_t lo, hi;
} job_t;

static void* worker(void* a) {
    job_t* j = (job_t*)a;
    for (uint64_t i = j->lo; i < j->hi; ++i)
        zpo_parse(j->arena + j->offs[i], j->lens[i], &j->recs[i], j->inner ? &j->inner[i] : 0);
    return 0;
}

/* Parses n frames with `nthreads` threads over contiguous shards
 * (nthreads <= 0: all online cores). Returns the thread count used. */
int zpo_parse_batch(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                    uint64_t n, zp_record* recs, zp_ext_offsets* inner, int nthreads) {
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads > 256) nthreads = 256;
    if (nthreads < 1) nthreads = 1;
    pthread_t th[256];
    int started[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (job_t){arena, offs, lens, recs, inner, n * t / nthreads, n * (t + 1) / nthreads};
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
                const zp_record* recs, uint64_t n, void* const* cols) {
    for (int c = 0; c < ZP_COL_COUNT; ++c)
        if (cols[c]) memset(cols[c], 0, n * (uint64_t)col_width[c]);
    for (uint64_t i = 0; i < n; ++i) {
        const zp_record* r = &recs[i];
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
