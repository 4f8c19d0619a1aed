/*
 * zero_packet.h — C ABI of the MI355X-native batched PacketParser::parse.
 *
 * This is the drop-in boundary for zero-packet's parse path
 * (/root/reference/src/packet/parser.rs:53). The reference has no FFI of its
 * own; its boundary is the Rust API
 *
 *     pub fn PacketParser::parse(bytes: &'a [u8]) -> Result<PacketParser<'a>, &'static str>
 *
 * whose result is nine `Option<Reader>` fields (parser.rs:22-32). Every
 * reader is a sub-slice `&frame[start..]` that runs to the end of the frame,
 * so a parsed packet is fully described by header START OFFSETS. One
 * zp_record per frame carries those offsets plus presence bits, so a caller
 * (C++ facade include/zero_packet.hpp, the Rust shim in INTEGRATION.md) can
 * rebuild every reader without re-parsing.
 *
 * Plain pointers and sizes only; no torch types. Device pointers are HIP
 * device memory; hipStream_t is passed as void*.
 */
#ifndef ZERO_PACKET_H
#define ZERO_PACKET_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZP_ABI_VERSION 6   /* 2: 16-B record, extension chains in the ext side array;
                              3: reader-accessor error codes 36-37 (ZP_ERR_COUNT 38,
                                 ZP_STATS_COUNT 62), standalone readers and the
                                 checksum primitives (zp_reader_new, zp_*checksum*);
                              4: 8-B record (flags word + packed offsets); the IPv6
                                 final next header of a chain in its ext entry;
                              5: the far-L4 form (Ethernet code 3, the whole L4
                                 offset in `offs`) replaces v4's saturation at
                                 ZP_L4_FAR; zp_rec_decode;
                              6: the inline outer chain (ZP_CHAIN_INLINE): a short
                                 RFC-ordered IPv6 extension chain of a frame without
                                 ip_in_ip lives in the record, no ext entry */

/* ------------------------------------------------------------------------- */
/* Per-packet parse error codes. One code per DISTINCT reference error string */
/* (identical strings collapse: icmpv4.rs:94 == icmpv6.rs:91). zp_err_str()   */
/* returns the exact reference string. Codes marked (unreachable) cannot be   */
/* produced by parse() because an earlier check subsumes them; they exist so  */
/* the per-reader views can report them.                                      */
/* ------------------------------------------------------------------------- */
typedef enum zp_err {
    ZP_OK = 0,
    ZP_ERR_ETH_FRAME_TOO_SHORT = 1,   /* parser.rs:160                          */
    ZP_ERR_ETH_SLICE_TOO_SHORT = 2,   /* ethernet.rs:143 (unreachable)          */
    ZP_ERR_ETH_VLAN_TOO_SHORT = 3,    /* ethernet.rs:160 (unreachable)          */
    ZP_ERR_ETH_QINQ_TOO_SHORT = 4,    /* ethernet.rs:167 (unreachable)          */
    ZP_ERR_ETH_INVALID_QINQ = 5,      /* ethernet.rs:172                        */
    ZP_ERR_ARP_TOO_SHORT = 6,         /* arp.rs:132 (unreachable)               */
    ZP_ERR_ARP_INVALID_OPER = 7,      /* parser.rs:176                          */
    ZP_ERR_IPV4_TOO_SHORT = 8,        /* ipv4.rs:140 (encapsulated levels only) */
    ZP_ERR_IPV4_VERSION = 9,          /* parser.rs:192                          */
    ZP_ERR_IPV4_IHL_TOO_SHORT = 10,   /* parser.rs:196                          */
    ZP_ERR_IPV4_HDR_TOO_LONG = 11,    /* parser.rs:200                          */
    ZP_ERR_IPV4_TOTAL_LENGTH = 12,    /* parser.rs:204                          */
    ZP_ERR_IPV4_CHECKSUM = 13,        /* parser.rs:208                          */
    ZP_ERR_IPV4_HDR_EXCEEDS = 14,     /* ipv4.rs:240,254 (unreachable)          */
    ZP_ERR_IPV6_TOO_SHORT = 15,       /* ipv6.rs:149 (encapsulated levels only) */
    ZP_ERR_IPV6_VERSION = 16,         /* parser.rs:226                          */
    ZP_ERR_EXT_HBH_NOT_FIRST = 17,    /* headers.rs:99-101                      */
    ZP_ERR_EXT_OPTIONS_TOO_SHORT = 18,/* options.rs:85                          */
    ZP_ERR_EXT_OPTIONS_EXCEEDS = 19,  /* options.rs:149                         */
    ZP_ERR_EXT_ROUTING_TOO_SHORT = 20,/* routing.rs:109                         */
    ZP_ERR_EXT_ROUTING_EXCEEDS = 21,  /* routing.rs:190                         */
    ZP_ERR_EXT_FRAGMENT_TOO_SHORT = 22,/* fragment.rs:99                        */
    ZP_ERR_EXT_AUTH_TOO_SHORT = 23,   /* authentication.rs:107                  */
    ZP_ERR_EXT_AUTH_EXCEEDS = 24,     /* authentication.rs:195                  */
    ZP_ERR_TCP_TOO_SHORT = 25,        /* tcp.rs:143                             */
    ZP_ERR_TCP_DATA_OFFSET = 26,      /* parser.rs:242                          */
    ZP_ERR_TCP_FLAGS = 27,            /* parser.rs:246                          */
    ZP_ERR_UDP_TOO_SHORT = 28,        /* udp.rs:105                             */
    ZP_ERR_UDP_LENGTH = 29,           /* parser.rs:262                          */
    ZP_ERR_ICMP_TOO_SHORT = 30,       /* icmpv4.rs:94 == icmpv6.rs:91           */
    ZP_ERR_ICMPV4_TYPE = 31,          /* parser.rs:278                          */
    ZP_ERR_ICMPV4_CODE = 32,          /* parser.rs:282                          */
    ZP_ERR_ICMPV6_TYPE = 33,          /* parser.rs:298                          */
    ZP_ERR_IPV4_L4_CHECKSUM = 34,     /* parser.rs:329                          */
    ZP_ERR_IPV6_L4_CHECKSUM = 35,     /* parser.rs:357                          */
    /* Errors of the reader accessors only (parse() never returns them):    */
    ZP_ERR_TCP_HDR_EXCEEDS = 36,      /* tcp.rs:227,239 (header()/payload())    */
    ZP_ERR_OPTIONS_DATA_EXCEEDS = 37, /* options.rs:115 (options())             */
    ZP_ERR_COUNT = 38
} zp_err;

/* ------------------------------------------------------------------------- */
/* Presence bits of zp_record.flags: the nine Option fields of PacketParser   */
/* (parser.rs:23-31) plus the IpInIp tag (misc.rs:6-9) and the two            */
/* Option<ExtensionHeaders> (ipv6.rs:140) with their six Option readers each  */
/* (headers.rs:20-25).                                                        */
/* ------------------------------------------------------------------------- */
#define ZP_F_ETHERNET      (1u << 0)
#define ZP_F_ARP           (1u << 1)
#define ZP_F_IPV4          (1u << 2)   /* outermost IPv4 (from Ethernet)        */
#define ZP_F_IPV6          (1u << 3)   /* outermost IPv6 (from Ethernet)        */
#define ZP_F_IP_IN_IP      (1u << 4)   /* first encapsulated IP header          */
#define ZP_F_IP_IN_IP_V6   (1u << 5)   /* ... and it is IpInIp::Ipv6            */
#define ZP_F_TCP           (1u << 6)
#define ZP_F_UDP           (1u << 7)
#define ZP_F_ICMPV4        (1u << 8)
#define ZP_F_ICMPV6        (1u << 9)
#define ZP_F_EXT           (1u << 10)  /* ipv6.extension_headers.is_some()      */
#define ZP_F_INNER_EXT     (1u << 11)  /* ip_in_ip IPv6 extension_headers Some  */
/* Extension header slots, in ExtensionHeaders field order (headers.rs:20-25). */
#define ZP_EXT_HBH   0
#define ZP_EXT_RT    1
#define ZP_EXT_FRAG  2
#define ZP_EXT_AH    3
#define ZP_EXT_DST1  4
#define ZP_EXT_DST2  5
#define ZP_EXT_SLOTS 6
#define ZP_F_EXT_SLOT(k)       (1u << (12 + (k)))  /* outer set, k in [0,6) */
#define ZP_F_INNER_EXT_SLOT(k) (1u << (18 + (k)))  /* inner set             */

/*
 * One parse result, 8 bytes (one dwordx2 store per frame). The record writes
 * are the only HBM writes of the parse, and writes mixed into the read
 * stream cost several times their bytes: the 8-B record took
 * 2-7 % off every configuration against the 16-B record of ABI v2/v3.
 *
 *   flags  bits  0-23  ZP_F_* presence and extension-slot bits (above)
 *          bits 24-25  Ethernet code: header length 14 + 4 * code (14 / 18 /
 *                      22, ethernet.rs:155-179); code 3 = the far-L4 form
 *          bits 26-31  err (zp_err; ZP_OK = 0)
 *   offs   bits  0-17  l4_off: start of the single tcp/udp/icmpv4/icmpv6 reader
 *          bits 18-31  inner_off: start of the ip_in_ip header (always below
 *                      16,384: Ethernet 22 + IPv6 40 + the longest chain 9,228)
 *
 * All offsets are FRAME offsets (bytes from the first byte of the frame).
 * ethernet/arp/ipv4/ipv6 start at offsets 0 / eth_len / eth_len / eth_len.
 * When err != ZP_OK the reference returns Err and no PacketParser exists:
 * the record is then zero except the err bits.
 *
 * Far-L4 form (ABI v5). An L4 reader that starts past ZP_L4_NEAR_MAX
 * (262,143) does not fit 18 bits; only an IPv6 jumbogram with thousands of
 * nested IPv6 headers reaches it (parser.rs:134-135 recurses without limit,
 * ipv6.rs:147-167 never checks payload_length). Its record carries Ethernet
 * code 3 and offs = the whole 32-bit L4 offset. The Ethernet header length
 * and inner_off, which such a frame always has (its first IP level ends by
 * byte 9,290), are then read from the frame, exactly as the parse found them:
 * eth_len by ethernet.rs:155-179, inner_off = eth_len + the outer IP header
 * (IPv4: IHL * 4; IPv6: 40 + extension_headers_len, the outer ext entry's
 * len). zp_rec_decode() does this; the facades call it. Every result stays
 * exact: nothing saturates.
 *
 * IPv6Reader::final_next_header() (ipv6.rs:219-227) is not in the record:
 * for an IPv6 header with an extension chain it is the chain's
 * final_next_header (headers.rs:26), stored in its zp_ext_offsets entry;
 * without a chain it is the header's next-header byte (frame offset ip + 6).
 */
typedef struct zp_record {
    uint32_t flags;
    uint32_t offs;
} zp_record;

#define ZP_F_MASK        0x00FFFFFFu
#define ZP_L4_NEAR_MAX   0x3FFFFu   /* largest l4_off of the ordinary form   */
#define ZP_ETH_CODE_FAR  3u         /* flags bits 24-25 of the far-L4 form   */
static inline uint32_t zp_rec_err(zp_record r)     { return r.flags >> 26; }
static inline int      zp_rec_is_far(zp_record r)  { return ((r.flags >> 24) & 3u) == ZP_ETH_CODE_FAR; }
static inline uint32_t zp_rec_l4_off(zp_record r)  { return zp_rec_is_far(r) ? r.offs : r.offs & ZP_L4_NEAR_MAX; }
/* Ordinary form only (0 for a far-L4 record: zp_rec_decode reads them from the frame). */
static inline uint32_t zp_rec_eth_len(zp_record r)   { return zp_rec_is_far(r) ? 0u : 14u + 4u * ((r.flags >> 24) & 3u); }
static inline uint32_t zp_rec_inner_off(zp_record r) {
    return zp_rec_is_far(r) || !(r.flags & ZP_F_IP_IN_IP) ? 0u : r.offs >> 18;
}

/*
 * Inline outer chain (ABI v6). A frame without an ip_in_ip header leaves the
 * inner_off field (offs bits 18-31) free. When its outer IPv6 extension chain
 * is short and in RFC 8200 order and the frame has an L4 reader, the chain is
 * stored there and its ext entry is NOT written (c4-shaped traffic then
 * writes 8 B per frame instead of 8 + 16):
 *
 *   offs bit 31      ZP_CHAIN_INLINE
 *   offs bits 18-20  Hop-by-Hop  length code c: (c + 1) * 8 B   (options.rs:123)
 *   offs bits 21-22  Destination 1st         c: (c + 1) * 8 B
 *   offs bits 23-25  Routing                 c: (c + 1) * 8 B   (routing.rs:164)
 *   (Fragment: always 8 B, fragment.rs:158)
 *   offs bits 26-27  Authentication          c: (c + 2) * 4 B   (authentication.rs:173)
 *   offs bits 28-29  Destination 2nd         c: (c + 1) * 8 B
 *
 * The present headers (the record's ZP_F_EXT_SLOT bits) lie back to back in
 * the order Hop-by-Hop, Destination 1st, Routing, Fragment, Authentication,
 * Destination 2nd; slot offsets are the running sums, extension_headers_len
 * the total, and final_next_header (headers.rs:26) the protocol of the
 * record's L4 reader (6 / 17 / 1 / 58). zp_rec_chain() rebuilds the
 * zp_ext_offsets entry; the host paths (zp_parse_batch_host, zp_parse_one,
 * the ring) hand out the rebuilt entry, so only device-batch callers see the
 * inline form. Any other chain keeps its 16-B entry.
 */
#define ZP_CHAIN_INLINE (1u << 31)
static inline int zp_rec_chain_inline(zp_record r) {
    return (r.flags >> 26) == 0 && !zp_rec_is_far(r) &&
           (r.flags & (ZP_F_EXT | ZP_F_IP_IN_IP)) == ZP_F_EXT && (r.offs & ZP_CHAIN_INLINE) != 0;
}

/*
 * One IPv6 extension chain (Some(ExtensionHeaders), headers.rs:19-28), 16 B:
 * len = IPv6Reader::extension_headers_len (ipv6.rs:141), off[k] = start of
 * slot k relative to the IPv6 payload (frame offset ip + 40 + off[k]),
 * final_nh = ExtensionHeaders::final_next_header (headers.rs:26).
 *
 * The ext side array of a batch of n frames holds 2n entries:
 *   ext[i]     the outer ipv6 chain of frame i, valid iff flags & ZP_F_EXT and
 *              the chain is not inline (zp_rec_chain_inline; device batches only);
 *   ext[n + i] the ip_in_ip IPv6 chain,           valid iff flags & ZP_F_INNER_EXT.
 * Entries whose flag is clear are unspecified (the kernel may leave them
 * untouched or zero them). Passing ext = NULL drops the chains (the records
 * still carry their presence and slot bits).
 */
typedef struct zp_ext_offsets {
    uint16_t len;
    uint16_t off[ZP_EXT_SLOTS];
    uint8_t  final_nh;
    uint8_t  reserved;
} zp_ext_offsets;

/* The zp_ext_offsets entry of an inline outer chain (zp_rec_chain_inline(r)
 * must hold): slot offsets, extension_headers_len and final_next_header. */
static inline void zp_rec_chain(zp_record r, zp_ext_offsets* x) {
    static const uint8_t order[6] = {ZP_EXT_HBH, ZP_EXT_DST1, ZP_EXT_RT, ZP_EXT_FRAG,
                                     ZP_EXT_AH, ZP_EXT_DST2};
    const uint32_t c = r.offs >> 18;
    const uint32_t len[6] = {                         /* by slot                   */
        ((c & 7u) + 1u) * 8u,                         /* ZP_EXT_HBH,  bits 18-20   */
        (((c >> 5) & 7u) + 1u) * 8u,                  /* ZP_EXT_RT,   bits 23-25   */
        8u,                                           /* ZP_EXT_FRAG               */
        (((c >> 8) & 3u) + 2u) * 4u,                  /* ZP_EXT_AH,   bits 26-27   */
        (((c >> 3) & 3u) + 1u) * 8u,                  /* ZP_EXT_DST1, bits 21-22   */
        (((c >> 10) & 3u) + 1u) * 8u};                /* ZP_EXT_DST2, bits 28-29   */
    uint32_t at = 0;
    for (int k = 0; k < ZP_EXT_SLOTS; ++k) x->off[k] = 0;
    for (int j = 0; j < 6; ++j) {
        const int k = order[j];
        if (r.flags & ZP_F_EXT_SLOT(k)) { x->off[k] = (uint16_t)at; at += len[k]; }
    }
    x->len = (uint16_t)at;
    x->final_nh = (uint8_t)((r.flags & ZP_F_TCP) ? 6 : (r.flags & ZP_F_UDP) ? 17
                          : (r.flags & ZP_F_ICMPV4) ? 1 : 58);
    x->reserved = 0;
}

/* A record with every field unpacked (PacketParser's readers by start
 * offset): flags = ZP_F_* bits, eth_len 14/18/22, final_nh / inner_final_nh
 * = IPv6Reader::final_next_header() (ipv6.rs:219-227) of the outer /
 * ip_in_ip IPv6 header (0 where absent); all zero but err on an error. */
typedef struct zp_rec_fields {
    uint32_t flags;
    uint8_t  err, eth_len, final_nh, inner_final_nh;
    uint32_t inner_off, l4_off;
} zp_rec_fields;

/* Unpacks `*rec`, the record of `frame` (len bytes), both forms (see above).
 * ext: NULL or the frame's two entries (outer chain, ip_in_ip chain); where
 * the record flags a chain and ext is NULL the chain is re-walked over the
 * frame (ipv6.rs:147-167), which gives the same values for a frame the
 * parse accepted. Host code. Returns 0, or -1 when the record cannot belong
 * to this frame (an offset past its end, a far record without an L4 reader
 * or an ip_in_ip header). */
int zp_rec_decode(const zp_record* rec, const uint8_t* frame, uint64_t len,
                  const zp_ext_offsets* ext, zp_rec_fields* out);

/* ------------------------------------------------------------------------- */
/* Library info                                                              */
/* ------------------------------------------------------------------------- */
/* Returns ZP_ABI_VERSION. */
int zp_abi_version(void);
/* Exact reference error string for a zp_err code ("" for ZP_OK, NULL if out
 * of range). Replaces the `&'static str` of Result (parser.rs:53). */
const char* zp_err_str(int code);
/* Last HIP error string seen by this library on the calling thread. */
const char* zp_last_error(void);

/* ------------------------------------------------------------------------- */
/* Batch parse — the hot path.                                                */
/* Replaces a loop of PacketParser::parse(&arena[off[i]..off[i]+len[i]])      */
/* (parser.rs:53) over n frames.                                              */
/* ------------------------------------------------------------------------- */
/*
 * Device-resident batch parse. All pointers are device memory on the current
 * HIP device; the call only enqueues work on `stream` (a hipStream_t, NULL =
 * default stream) and returns. Frames may lie anywhere in `arena` (gaps,
 * overlaps and any order are allowed); the fast path is taken for the common
 * packed, increasing layout. `ext` (2n entries, see zp_ext_offsets) may be
 * NULL. Returns 0 on success or
 * a negative value if the launch failed (see zp_last_error()).
 * Precondition (not checked on the device: the descriptors live in HBM and the
 * call does not synchronise): offs[i] + lens[i] <= the arena's size for every
 * i. A descriptor past the arena reads past the allocation and faults the
 * GPU. The Python wrapper (batch.parse_batch) checks this with one device
 * reduction unless told not to.
 */
int zp_parse_batch_device(const uint8_t* arena, const uint64_t* offs,
                          const uint32_t* lens, uint64_t n,
                          zp_record* records, zp_ext_offsets* ext,
                          void* stream);

/*
 * Record codes (round 6). Inside the parse's read stream a record store
 * costs in proportion to the contiguous bytes a wave stores,
 * so a full tile of 64 frames whose records all have the common form (no
 * error, no IP-in-IP, no extension headers, the L4 reader right after a
 * 20-B IPv4 or 40-B IPv6 header: config 3) is stored as one code byte per
 * frame over the tile's first 8 records, and a second kernel on the same
 * stream rewrites the tile's 64 records from the codes. The records a
 * caller reads are the same either way (zp_parse_batch_device still only
 * enqueues). mode 0: automatic (batches of at least 2,097,152 frames
 * whose traffic has code tiles: probe calls, one per 16 calls per device
 * and one at every change of batch size, tell, through a mapped host word
 * their second kernel sets and an event queried without waiting), 1:
 * always, 2: never. Process-wide; returns the previous mode, or -1 for an
 * unknown mode.
 */
int zp_set_record_slots(int mode);
/* The automatic mode's current decision on the calling thread's device for
 * batches of at least 2,097,152 frames (1: record codes, 0: one kernel);
 * the latest completed probe's verdict, 1 before any. For reports. */
int zp_record_slots_state(void);

/* Host-buffer convenience path: the frames, descriptors and outputs live in
 * host memory (a NIC ring / raw socket buffer). Stages through pinned buffers
 * and overlaps H2D copy, parse and D2H copy in chunks on `ctx`'s streams.
 * Synchronous. Returns 0 on success, negative on HIP failure.
 * A zp_ctx owns pinned staging buffers, device buffers and streams: it must
 * not be used by two host threads at once (one context per thread, or a
 * lock around every call that takes it, as the Python facade does). */
typedef struct zp_ctx zp_ctx;
zp_ctx* zp_ctx_create(int device, uint64_t chunk_bytes);
void    zp_ctx_destroy(zp_ctx* ctx);
int zp_parse_batch_host(zp_ctx* ctx, const uint8_t* arena, uint64_t arena_bytes,
                        const uint64_t* offs, const uint32_t* lens, uint64_t n,
                        zp_record* records, zp_ext_offsets* ext);
/* The same over several devices (one context each, e.g. the 8 GPUs of a
 * node): contiguous frame ranges with balanced byte totals run concurrently,
 * one host thread per context. No cross-device exchange. Returns 0 or the
 * first failing context's code (zp_last_error() names the context). */
int zp_parse_batch_host_multi(zp_ctx* const* ctxs, int nctx, const uint8_t* arena,
                              uint64_t arena_bytes, const uint64_t* offs,
                              const uint32_t* lens, uint64_t n, zp_record* records,
                              zp_ext_offsets* ext);
/* One frame through the GPU path (PacketParser::parse equivalent,
 * parser.rs:53). ext: NULL or 2 entries (outer, ip_in_ip chain; zeroed where
 * the record flags no chain). Returns the zp_err code (>= 0) or a negative
 * value on HIP failure. The frame is copied into ctx's mapped pinned block;
 * by default the device's shared resident server (one kernel per device and
 * process, one wave per context, launched on demand) polls a doorbell there,
 * parses the frame in place and writes the record back: no kernel launch per
 * call. The kernel leaves after 1 ms resident whatever
 * the traffic; the next call replaces it (under steady traffic a caller
 * queues the next one and retires the old one). A device-wide
 * synchronisation (hipDeviceSynchronize, torch.cuda.synchronize, hipFree)
 * issued meanwhile waits for the running kernel, so about 1 ms at most;
 * zp_parse_one_config stops it at once. Frames over 64 KiB take the batch
 * host path. Like every zp_ctx call, one thread at a time per ctx (one
 * context per thread, or a pool); contexts of one device share the server,
 * so their calls run concurrently. */
int zp_parse_one(zp_ctx* ctx, const uint8_t* frame, uint64_t len,
                 zp_record* record, zp_ext_offsets ext[2]);
/* zp_parse_one's mode on ctx: idle_us > 0 = the device's resident server
 * (the default, 5000; the value is no longer a timeout: the server's life is
 * 1 ms); 0 = one batch-kernel launch and a stream wait per call (~18 us).
 * Stops the device's server either way (every context's next call
 * relaunches it). Returns 0, or -1 on a NULL ctx. */
int zp_parse_one_config(zp_ctx* ctx, uint32_t idle_us);
/* The calling thread's current HIP device (hipGetDevice), -1 on failure:
 * the device a facade creates its contexts on. */
int zp_device_current(void);

/* ------------------------------------------------------------------------- */
/* Standalone readers and the checksum primitives.                           */
/* The reference's second usage (README.md:110-115) builds a reader directly */
/* over a slice: TcpReader::new(&packet[off..])? and reads its fields. Every  */
/* reader's `new` is a checked constructor returning Result (the minimum     */
/* slice length; Ethernet also the VLAN tagging; IPv6 also the extension    */
/* walk, ipv6.rs:159). These are host-side views over host bytes, like the  */
/* reference's: one slice, no batch, no device. The batch parse stays the   */
/* device path above.                                                        */
/* ------------------------------------------------------------------------- */
typedef enum zp_reader_kind {
    ZP_READER_ETHERNET = 0,  /* EthernetReader::new               ethernet.rs:141 */
    ZP_READER_ARP = 1,       /* ArpReader::new                    arp.rs:130      */
    ZP_READER_IPV4 = 2,      /* IPv4Reader::new                   ipv4.rs:138     */
    ZP_READER_IPV6 = 3,      /* IPv6Reader::new (+ extension walk) ipv6.rs:147-167 */
    ZP_READER_OPTIONS = 4,   /* OptionsHeaderReader::new          options.rs:83   */
    ZP_READER_ROUTING = 5,   /* RoutingHeaderReader::new          routing.rs:107  */
    ZP_READER_FRAGMENT = 6,  /* FragmentHeaderReader::new         fragment.rs:97  */
    ZP_READER_AUTH = 7,      /* AuthenticationHeaderReader::new   authentication.rs:105 */
    ZP_READER_TCP = 8,       /* TcpReader::new                    tcp.rs:141      */
    ZP_READER_UDP = 9,       /* UdpReader::new                    udp.rs:103      */
    ZP_READER_ICMPV4 = 10,   /* Icmpv4Reader::new                 icmpv4.rs:92    */
    ZP_READER_ICMPV6 = 11,   /* Icmpv6Reader::new                 icmpv6.rs:89    */
    ZP_READER_KIND_COUNT = 12
} zp_reader_kind;

/* What a successful constructor computed besides the slice itself. */
typedef struct zp_reader_info {
    uint32_t header_len;     /* Ethernet: 14/18/22 (calculate_header_len,      */
                             /* ethernet.rs:155-179); 0 for the other kinds    */
    uint32_t flags;          /* IPv6: ZP_F_EXT when extension_headers is Some, */
                             /* ZP_F_EXT_SLOT(k) per present slot; else 0      */
    uint8_t  final_nh;       /* IPv6: final_next_header() (ipv6.rs:219-227)    */
    uint8_t  reserved[3];
    zp_ext_offsets ext;      /* IPv6: extension_headers_len (ext.len) and the  */
                             /* slot offsets, relative to the IPv6 payload     */
} zp_reader_info;

/* XReader::new(&bytes[..len]) of reader `kind`. Returns ZP_OK (info filled,
 * when not NULL) or the zp_err code of the reference's Err, whose string is
 * zp_err_str(code); -1 for an unknown kind or bytes == NULL with len > 0. */
int zp_reader_new(int kind, const uint8_t* bytes, uint64_t len, zp_reader_info* info);

/* internet_checksum(data, accumulator) (checksum.rs:5-29): RFC 1071 sum of
 * the big-endian 16-bit words (an odd tail byte as the high byte) with u32
 * wrap-around, folded, complemented. */
uint16_t zp_internet_checksum(const uint8_t* data, uint64_t len, uint32_t accumulator);
/* verify_internet_checksum (checksum.rs:33-35): 1 if the checksum is 0. */
int zp_verify_internet_checksum(const uint8_t* data, uint64_t len, uint32_t accumulator);
/* pseudo_header(src, dest, protocol, length) (checksum.rs:38-69) for 4-byte
 * (IPv4) or 16-byte (IPv6) addresses: the address words + protocol +
 * (u32)length. addr_len other than 4 or 16 returns 0. */
uint32_t zp_pseudo_header(const uint8_t* src, const uint8_t* dest, uint32_t addr_len,
                          uint8_t protocol, uint64_t length);

/* ------------------------------------------------------------------------- */
/* Per-batch counters: frames per presence bit of          */
/* zp_record.flags and frames per zp_err code, for monitoring a capture      */
/* (protocol mix, error histogram) without copying the records to the host. */
/* ------------------------------------------------------------------------- */
#define ZP_STATS_FLAG_BITS 24                      /* flags bits 0-23 (ZP_F_*, slots) */
#define ZP_STAT_FLAG(bit)  (bit)                   /* frames with flags bit `bit` set */
#define ZP_STAT_ERR(code)  (ZP_STATS_FLAG_BITS + (code))  /* frames with err == code   */
#define ZP_STATS_COUNT     (ZP_STATS_FLAG_BITS + ZP_ERR_COUNT)
/* Adds the counts of records[0, n) into counts[ZP_STATS_COUNT] (device u64,
 * zeroed by the caller; several batches accumulate). Enqueues on `stream`.
 * The counts of several devices add up on the host (frames are independent).
 * Returns 0 or negative on launch failure. */
int zp_stats_device(const zp_record* records, uint64_t n, uint64_t* counts, void* stream);

/* Diagnostic: one plain streaming read of bytes [p, p + bytes) (device
 * memory, 16-B aligned; the tail below 16 B is not read), enqueued on
 * `stream`. bench.py times it over the arena beside the parse: the parse's
 * rate moves with the physical placement of the arena and so
 * does a pure read, which tells placements apart. sink: one device u32
 * (practically never written). Returns 0 or negative. */
int zp_probe_read_device(const uint8_t* p, uint64_t bytes, uint32_t* sink, void* stream);
/* Diagnostic: the parse kernel's memory traffic without its work. Over
 * ceil(n / 64) waves (one per workgroup, with a parse wave's LDS, so at its
 * occupancy) wave t loads descriptors offs / lens [64 t, 64 t + 64) ∩ [0, n)
 * (when both are given), streams the t-th equal slice of [p, p + bytes) and
 * then, when records != NULL, stores the 8-B words records[64 t, 64 t + 64)
 * ∩ [0, n) (their contents are junk), as the parse does per tile. bench.py
 * times it over the bench's own arena, descriptors and records
 * (roofline.placement). Returns 0 or negative. */
int zp_probe_tiles_device(const uint8_t* p, uint64_t bytes, uint64_t n, const uint64_t* offs,
                          const uint32_t* lens, zp_record* records, uint32_t* sink,
                          void* stream);
/* Diagnostic: the same pattern with record codes (zp_set_record_slots): a
 * full tile stores one byte per frame instead of its 8-B records and the
 * parse's expansion kernel then rewrites records [0, n) (junk contents). */
int zp_probe_tiles_codes_device(const uint8_t* p, uint64_t bytes, uint64_t n,
                                const uint64_t* offs, const uint32_t* lens, zp_record* records,
                                uint32_t* sink, void* stream);

/* ------------------------------------------------------------------------- */
/* Host-ring ingestion pipeline. Frames start in host */
/* memory (a NIC ring / raw socket, README.md:85-115 of the reference). A     */
/* ring holds `nslots` slots, each with pinned host buffers, device buffers   */
/* and its own stream. The producer acquires a slot, fills its arena and      */
/* descriptors in place (a NIC would DMA straight into the pinned arena) and  */
/* submits it; the slot then runs H2D -> parse -> D2H asynchronously while    */
/* the next slot fills. The consumer takes completed slots in submission      */
/* order (wait / poll), reads the records and releases the slot.              */
/* Slot states: FREE -acquire-> FILLING -submit-> IN_FLIGHT -wait/poll->      */
/* DONE -release-> FREE. One producer and one consumer thread may use a ring  */
/* concurrently. All functions return 0 on success, negative on error (see    */
/* zp_last_error()), ZP_RING_TIMEOUT when a wait expires.                     */
/* ------------------------------------------------------------------------- */
typedef struct zp_ring zp_ring;
#define ZP_RING_TIMEOUT (-4)
typedef struct zp_ring_slot {
    int32_t id;                         /* slot index                          */
    uint8_t* arena;                     /* pinned host arena, arena_cap bytes  */
    uint64_t* offs;                     /* pinned frame offsets into arena     */
    uint32_t* lens;                     /* pinned frame lengths                */
    uint64_t arena_cap, frames_cap;
    const zp_record* records;           /* results (valid after wait/poll)     */
    const zp_ext_offsets* ext;          /* 2n entries (zp_ext_offsets), n below */
    uint64_t n;                         /* frames in the slot (after wait/poll) */
    uint64_t seq;                       /* submission sequence number          */
} zp_ring_slot;

zp_ring* zp_ring_create(int device, uint32_t nslots, uint64_t slot_bytes,
                        uint64_t slot_frames);
void zp_ring_destroy(zp_ring* ring);
/* Hands out the next slot (in ring order) once it is FREE, as FILLING.
 * timeout_ms < 0 blocks, 0 only checks; ZP_RING_TIMEOUT when it expires. */
int zp_ring_acquire(zp_ring* ring, zp_ring_slot* slot, int64_t timeout_ms);
/* Enqueues H2D + parse + D2H for the first n frames of an acquired slot.
 * Frames must lie inside the slot arena (else -1, nothing enqueued). */
int zp_ring_submit(zp_ring* ring, int32_t id, uint64_t n);
/* Hands out the oldest submitted slot once its records are in host memory.
 * timeout_ms < 0 blocks, 0 polls; ZP_RING_TIMEOUT when nothing is ready. */
int zp_ring_wait(zp_ring* ring, zp_ring_slot* slot, int64_t timeout_ms);
/* Returns a DONE slot to the producer. */
int zp_ring_release(zp_ring* ring, int32_t id);

/* ------------------------------------------------------------------------- */
/* Column views: the reader getters of every parsed  */
/* frame gathered into SoA device columns, so downstream consumers get ready */
/* columns (5-tuple, VLAN TCIs, flow label ...) without a host pass.         */
/* Entry i of a column is 0 when record i holds an error or the reader the   */
/* column belongs to is absent. Multi-byte integers are host order (LE);     */
/* byte-array columns (MACs, addresses) are the frame bytes as they stand.   */
/* "outer IP" = PacketParser::ipv4 / ::ipv6, "inner IP" = ::ip_in_ip.        */
/* ------------------------------------------------------------------------- */
typedef enum zp_col {
    ZP_COL_DEST_MAC = 0,     /* u8[6]  EthernetReader::dest_mac (ethernet.rs:195-198)     */
    ZP_COL_SRC_MAC,          /* u8[6]  EthernetReader::src_mac (ethernet.rs:201-204)      */
    ZP_COL_ETHERTYPE,        /* u16    EthernetReader::ethertype (ethernet.rs:209-212)    */
    ZP_COL_VLAN_TCI,         /* u16    vlan_tag().1, or double_vlan_tag().0.1 (:218-244)  */
    ZP_COL_VLAN_INNER_TCI,   /* u16    double_vlan_tag().1.1 (ethernet.rs:232-244)        */
    ZP_COL_ARP_OPER,         /* u16    ArpReader::oper (arp.rs:174-177)                   */
    ZP_COL_IP_VERSION,       /* u8     4 or 6 when the outer IP reader is present         */
    ZP_COL_SRC_ADDR,         /* u8[16] IPv4Reader::src_ip in bytes 0-3 (ipv4.rs:210-213)  */
                             /*        or IPv6Reader::src_addr (ipv6.rs:245-248)          */
    ZP_COL_DEST_ADDR,        /* u8[16] dest_ip (ipv4.rs:216-219) / dest_addr (ipv6.rs:253-256) */
    ZP_COL_PROTOCOL,         /* u8     IPv4 protocol (ipv4.rs:204-207) / IPv6             */
                             /*        final_next_header (ipv6.rs:219-227)                */
    ZP_COL_TTL,              /* u8     ttl (ipv4.rs:198-201) / hop_limit (ipv6.rs:237-240) */
    ZP_COL_TOS,              /* u8     dscp<<2|ecn (ipv4.rs:160-169) / traffic_class (ipv6.rs:181) */
    ZP_COL_IP_ID,            /* u32    IPv4 id (ipv4.rs:180) / flow_label (ipv6.rs:189)    */
    ZP_COL_IP_LEN,           /* u16    total_length (ipv4.rs:174) / payload_length (ipv6.rs:199)*/
    ZP_COL_INNER_VERSION,    /* u8     4 or 6 when ip_in_ip is present (misc.rs:6-9)      */
    ZP_COL_INNER_SRC_ADDR,   /* u8[16] as ZP_COL_SRC_ADDR, of the ip_in_ip reader         */
    ZP_COL_INNER_DEST_ADDR,  /* u8[16]                                                    */
    ZP_COL_INNER_PROTOCOL,   /* u8     protocol / final_next_header of ip_in_ip           */
    ZP_COL_L4_PROTO,         /* u8     6 tcp, 17 udp, 1 icmpv4, 58 icmpv6; 0 none         */
    ZP_COL_SRC_PORT,         /* u16    TcpReader / UdpReader::src_port (tcp.rs:151, udp.rs:113) */
    ZP_COL_DEST_PORT,        /* u16    dest_port (tcp.rs:157, udp.rs:119)                 */
    ZP_COL_TCP_SEQ,          /* u32    sequence_number (tcp.rs:163-170)                   */
    ZP_COL_TCP_ACK,          /* u32    ack_number (tcp.rs:172-179)                        */
    ZP_COL_TCP_FLAGS,        /* u8     flags (tcp.rs:193-196)                             */
    ZP_COL_TCP_WINDOW,       /* u16    window_size (tcp.rs:199-202)                       */
    ZP_COL_ICMP_TYPE,        /* u8     icmp_type (icmpv4.rs:102, icmpv6.rs:99)            */
    ZP_COL_ICMP_CODE,        /* u8     icmp_code (icmpv4.rs:108, icmpv6.rs:105)           */
    ZP_COL_L4_CHECKSUM,      /* u16    checksum() (tcp.rs:205, udp.rs:125, icmpv4.rs:114) */
    ZP_COL_PAYLOAD_OFF,      /* u32    frame offset of the L4 reader's payload(); 0 when  */
                             /*        absent or when payload() returns Err (tcp.rs:235-243) */
    ZP_COL_COUNT
} zp_col;

/* Element size in bytes of column `col` (0 if out of range). */
int zp_col_width(int col);

/* Fills the requested columns for n parsed frames: cols[c] is a device array
 * of n * zp_col_width(c) bytes, or NULL to skip column c. arena/offs/lens are
 * the batch given to zp_parse_batch_device, records its output (device
 * memory). Enqueues on `stream`; returns 0 or negative on launch failure. */
int zp_extract_columns_device(const uint8_t* arena, const uint64_t* offs,
                              const uint32_t* lens, const zp_record* records, uint64_t n,
                              void* const* cols, void* stream);

/* zp_parse_batch_device and zp_extract_columns_device fused: one pass over
 * the frames writes the records and the requested columns (read from the
 * parse kernel's staged header window; cols as above, NULL entries skipped).
 * Same results as the two calls in sequence. */
int zp_parse_batch_columns_device(const uint8_t* arena, const uint64_t* offs,
                                  const uint32_t* lens, uint64_t n, zp_record* records,
                                  zp_ext_offsets* ext, void* const* cols, void* stream);

/* ------------------------------------------------------------------------- */
/* Batched PacketBuilder. The reference builds one    */
/* frame with a typestate chain over a caller-sized buffer                    */
/* (builder.rs:55-909): PacketBuilder::new(&mut buf).ethernet(..).ipv4(..)    */
/* .tcp(..).build(). Here every frame of a batch carries its chain as a run   */
/* of zp_build_op (one op per builder method, in call order) and the kernel   */
/* executes all chains in place over the frames' buffers, with the writers'   */
/* exact byte semantics: read-modify-write of shared bytes, checksums over    */
/* the whole remaining buffer, and the first Err stopping the chain with the  */
/* partial writes left in place, as the reference leaves them.                */
/* A chain that the typestate graph (builder.rs:817-909) would not compile    */
/* is refused before anything is written (ZP_BERR_TRANSITION); a chain whose  */
/* reference run would panic reports ZP_BERR_PANIC.                           */
/* ------------------------------------------------------------------------- */
typedef enum zp_build_kind {
    ZP_B_ETHERNET = 1,       /* builder.rs:113  src=src_mac dst=dest_mac h0=ethertype      */
    ZP_B_ETHERNET_VLAN = 2,  /* builder.rs:141  + h1=tci                                    */
    ZP_B_ETHERNET_QINQ = 3,  /* builder.rs:171  + h1=tci1 h2=tci2                           */
    ZP_B_ARP = 4,            /* builder.rs:203  h0=htype h1=ptype b0=hlen b1=plen h2=oper   */
                             /*   src[0:6]=sha src[6:10]=spa dst[0:6]=tha dst[6:10]=tpa      */
    ZP_B_IPV4 = 5,           /* builder.rs:248/343 b0=version b1=ihl b2=dscp b3=ecn          */
                             /*   h0=total_length h1=identification b4=flags h2=fragment_offset */
                             /*   b5=ttl b6=protocol src[0:4]=src_ip dst[0:4]=dest_ip          */
    ZP_B_IPV6 = 6,           /* builder.rs:300/395 b0=version b1=traffic_class w0=flow_label */
                             /*   h0=payload_length b2=next_header b3=hop_limit src dst      */
    ZP_B_HOP_BY_HOP = 7,     /* builder.rs:611  b0=next_header b1=extension_len data=options */
    ZP_B_DEST_OPTS1 = 8,     /* builder.rs:643  as hop_by_hop                               */
    ZP_B_ROUTING = 9,        /* builder.rs:675  b0=next_header b1=header_ext_len            */
                             /*   b2=routing_type b3=segments_left data=data                 */
    ZP_B_FRAGMENT = 10,      /* builder.rs:711  b0=next_header h0=fragment_offset b1=m_flag */
                             /*   w0=identification                                          */
    ZP_B_AUTH = 11,          /* builder.rs:747  b0=next_header b1=payload_len w0=spi        */
                             /*   w1=seq_num data=auth_data                                  */
    ZP_B_DEST_OPTS2 = 12,    /* builder.rs:785  as hop_by_hop                               */
    ZP_B_TCP = 13,           /* builder.rs:438  src/dst = pseudo-header addresses (4 B      */
                             /*   under IPv4 states, 16 B otherwise) h0=src_port h1=dest_port */
                             /*   w0=sequence_number w1=acknowledgment_number b0=data_offset  */
                             /*   b1=reserved b2=flags h2=window_size h3=urgent_pointer      */
                             /*   data=payload (optional)                                    */
    ZP_B_UDP = 14,           /* builder.rs:492  src/dst h0=src_port h1=dest_port h2=length  */
                             /*   data=payload (optional)                                    */
    ZP_B_ICMPV4 = 15,        /* builder.rs:534  b0=icmp_type b1=icmp_code data=payload (opt) */
    ZP_B_ICMPV6 = 16,        /* builder.rs:571  src/dst b0=icmp_type b1=icmp_code data (opt) */
    ZP_B_KIND_COUNT = 17
} zp_build_kind;

#define ZP_BUILD_NO_DATA 0xFFFFFFFFu   /* data_len: payload None (others: empty)   */

typedef struct zp_build_op {           /* 64 bytes */
    uint8_t  kind;                     /* zp_build_kind                            */
    uint8_t  b[7];
    uint16_t h[4];
    uint32_t w[2];
    uint32_t data_off;                 /* variable bytes at data + data_off        */
    uint32_t data_len;                 /* ... their length, or ZP_BUILD_NO_DATA    */
    uint8_t  src[16];
    uint8_t  dst[16];
} zp_build_op;

typedef enum zp_build_err {
    ZP_BUILD_OK = 0,
    ZP_BERR_ETH_SLICE = 1,            /* ethernet.rs:30                            */
    ZP_BERR_ETH_VLAN = 2,             /* ethernet.rs:85                            */
    ZP_BERR_ETH_QINQ = 3,             /* ethernet.rs:112                           */
    ZP_BERR_ARP_DATA = 4,             /* builder.rs:216                            */
    ZP_BERR_ARP_SLICE = 5,            /* arp.rs:17                                 */
    ZP_BERR_IPV4_DATA = 6,            /* builder.rs:264,359                        */
    ZP_BERR_IPV4_SLICE = 7,           /* ipv4.rs:18                                */
    ZP_BERR_IPV6_DATA = 8,            /* builder.rs:312,407                        */
    ZP_BERR_IPV6_SLICE = 9,           /* ipv6.rs:18                                */
    ZP_BERR_TCP_DATA = 10,            /* builder.rs:454                            */
    ZP_BERR_TCP_SLICE = 11,           /* tcp.rs:17                                 */
    ZP_BERR_TCP_PAYLOAD = 12,         /* tcp.rs:110 == udp.rs:84                   */
    ZP_BERR_UDP_DATA = 13,            /* builder.rs:502                            */
    ZP_BERR_UDP_SLICE = 14,           /* udp.rs:17                                 */
    ZP_BERR_ICMPV4_DATA = 15,         /* builder.rs:541                            */
    ZP_BERR_ICMP_SLICE = 16,          /* icmpv4.rs:20 == icmpv6.rs:17              */
    ZP_BERR_ICMPV4_PAYLOAD = 17,      /* icmpv4.rs:61                              */
    ZP_BERR_ICMPV6_DATA = 18,         /* builder.rs:580                            */
    ZP_BERR_ICMPV6_PAYLOAD = 19,      /* icmpv6.rs:58                              */
    ZP_BERR_HBH_DATA = 20,            /* builder.rs:618                            */
    ZP_BERR_DEST_DATA = 21,           /* builder.rs:650,792                        */
    ZP_BERR_OPTIONS_SLICE = 22,       /* options.rs:18                             */
    ZP_BERR_OPTIONS_MIN = 23,         /* options.rs:54                             */
    ZP_BERR_OPTIONS_MATCH = 24,       /* options.rs:60                             */
    ZP_BERR_OPTIONS_EXCEED = 25,      /* options.rs:67                             */
    ZP_BERR_ROUTING_DATA = 26,        /* builder.rs:684,719 (fragment_header too)  */
    ZP_BERR_ROUTING_SLICE = 27,       /* routing.rs:16                             */
    ZP_BERR_ROUTING_MIN = 28,         /* routing.rs:77                             */
    ZP_BERR_ROUTING_MATCH = 29,       /* routing.rs:83                             */
    ZP_BERR_ROUTING_EXCEED = 30,      /* routing.rs:90                             */
    ZP_BERR_AUTH_DATA = 31,           /* builder.rs:756                            */
    ZP_BERR_AUTH_SLICE = 32,          /* authentication.rs:16                      */
    ZP_BERR_AUTH_EXCEED = 33,         /* authentication.rs:88                      */
    ZP_BERR_PANIC = 34,               /* the reference would panic: fragment.rs:16 */
                                      /* panic!, or a slice index out of range      */
                                      /* (ipv4.rs:123, tcp.rs:114)                  */
    ZP_BERR_TRANSITION = 35,          /* chain not allowed by builder.rs:817-909    */
    ZP_BERR_COUNT = 36
} zp_build_err;

typedef struct zp_build_result {
    uint32_t header_len;               /* PacketBuilder::header_len() (builder.rs:65) */
    uint8_t  err;                      /* zp_build_err                             */
    uint8_t  ops_done;                 /* ops that returned Ok                     */
    uint16_t reserved;
} zp_build_result;

/* Exact reference string of a zp_build_err ("" for OK, NULL out of range). */
const char* zp_build_err_str(int code);

/* Runs n builder chains in place on the device. Frame i is the buffer
 * arena[offs[i] .. offs[i] + lens[i]) (the reference's `&mut [u8]`), its
 * chain is ops[op_start[i] .. op_start[i + 1]) (op_start has n + 1 entries),
 * variable bytes come from `data`. results may be NULL. All pointers are
 * device memory; enqueues on `stream`. Returns 0 or negative on failure.
 * Precondition (not checked on the device, as for zp_parse_batch_device):
 * every frame lies inside the arena, the frames do not overlap (the kernel
 * writes them), every op's data range lies inside `data`. The Python API
 * (BuildBatch.run) checks the descriptors first. */
int zp_build_batch_device(uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                          uint64_t n, const zp_build_op* ops, const uint32_t* op_start,
                          const uint8_t* data, zp_build_result* results, void* stream);

/* The same over host buffers (a transmit ring), through `ctx`: the frames'
 * bytes go H2D, the chains run, the frame bytes come back. data_bytes is the
 * size of the data blob. Synchronous. Returns 0 or negative on failure. */
int zp_build_batch_host(zp_ctx* ctx, uint8_t* arena, uint64_t arena_bytes,
                        const uint64_t* offs, const uint32_t* lens, uint64_t n,
                        const zp_build_op* ops, const uint32_t* op_start,
                        const uint8_t* data, uint64_t data_bytes, zp_build_result* results);

/* ------------------------------------------------------------------------- */
/* Synthetic batch generator (BASELINE.json configs 1-5, mixed config 6),    */
/* built from the builder's checksum-fill semantics                          */
/* (builder.rs:473-474,515-516,553,592-593).                                 */
/* Deterministic per packet: packet i depends only on (config, seed, i).      */
/* ------------------------------------------------------------------------- */
#define ZP_CFG_C1_ETH_IPV4_UDP_64 1  /* == C2 layout, CPU plumbing            */
#define ZP_CFG_C2_ETH_IPV4_UDP_64 2
#define ZP_CFG_C3_IPV4_MIX        3
#define ZP_CFG_C4_IPV6_EXT_VLAN   4
#define ZP_CFG_C5_IMIX_IPINIP     5
#define ZP_CFG_C6_MIXED           6  /* not a BASELINE config: per packet the shape
                                        of C3, C4 or C5 (5/16 each) or a 64-B ARP
                                        frame (1/16), so every tile mixes stacks */
#define ZP_GEN_SEED_DEFAULT 0x5EED2025ull

/* Frame length of packet `first + i`, i in [0, n), into d_lens (device). */
int zp_gen_lengths_device(int config, uint64_t seed, uint64_t first, uint64_t n,
                          uint32_t* lens, void* stream);
/* Writes frame `first + i` at arena + offs[i] (offs/lens device arrays as
 * produced by zp_gen_lengths_device + an exclusive scan). */
int zp_gen_frames_device(int config, uint64_t seed, uint64_t first, uint64_t n,
                         uint8_t* arena, const uint64_t* offs,
                         const uint32_t* lens, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* ZERO_PACKET_H */
