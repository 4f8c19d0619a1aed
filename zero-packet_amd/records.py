"""zp_record layout (include/zero_packet.h, ABI v6) as numpy dtypes."""
import ctypes

import numpy as np

# The 8-B record: flags (bits 0-23 ZP_F_*, 24-25 Ethernet code, 26-31 err)
# and offs (bits 0-17 l4_off, 18-31 inner_off when ZP_F_IP_IN_IP is set).
# unpack() gives the fields.
# Inline outer chain (ABI v6, ZP_CHAIN_INLINE): a frame without an ip_in_ip
# header may carry its short RFC-ordered outer IPv6 extension chain in offs
# bits 18-31 instead (bit 31 set, a 2-3-bit length code per header; no ext
# entry is written): chain_inline() / inline_chains().
# Far-L4 form (Ethernet code 3): offs is the whole L4 offset; the Ethernet
# header length and inner_off are read from the frame (decode()).
RECORD_DTYPE = np.dtype([("flags", "<u4"), ("offs", "<u4")])
assert RECORD_DTYPE.itemsize == 8
# unpack()'s per-field view (the final next headers are not in the record:
# ext entry of a chain, else the IPv6 next-header byte)
FIELDS_DTYPE = np.dtype([("flags", "<u4"), ("err", "u1"), ("eth_len", "u1"),
                         ("inner_off", "<u4"), ("l4_off", "<u4")])
F_MASK = 0x00FFFFFF
L4_NEAR_MAX = 0x3FFFF     # ZP_L4_NEAR_MAX: largest l4_off of the ordinary form
ETH_CODE_FAR = 3          # ZP_ETH_CODE_FAR
# One IPv6 extension chain (zp_ext_offsets). A batch of n frames has 2n of
# them: [0, n) the outer ipv6 chains, [n, 2n) the ip_in_ip ones; numpy views
# them as shape (2, n). final_nh = ExtensionHeaders::final_next_header.
EXT_DTYPE = np.dtype([("len", "<u2"), ("off", "<u2", (6,)), ("final_nh", "u1"),
                      ("reserved", "u1")])
assert EXT_DTYPE.itemsize == 16
RECORD_BYTES, EXT_BYTES = 8, 16


def unpack(rec):
    """RECORD_DTYPE array (or raw uint8 [n, 8]) -> FIELDS_DTYPE array. A
    far-L4 record gives its whole l4_off and eth_len = inner_off = 0 (they
    are in the frame, not the record: decode())."""
    rec = np.asarray(rec)
    if rec.dtype != RECORD_DTYPE:
        rec = np.ascontiguousarray(rec, dtype=np.uint8).view(RECORD_DTYPE).reshape(-1)
    w, o = rec["flags"].astype(np.uint32), rec["offs"].astype(np.uint32)
    out = np.zeros(w.shape, FIELDS_DTYPE)
    err = w >> 26
    out["err"] = err
    ok = err == 0
    far = ok & (((w >> 24) & 3) == ETH_CODE_FAR)
    near = ok & ~far
    out["flags"] = np.where(ok, w & F_MASK, 0)
    out["eth_len"] = np.where(near, 14 + 4 * ((w >> 24) & 3), 0)
    out["l4_off"] = np.where(near, o & L4_NEAR_MAX, np.where(far, o, 0))
    out["inner_off"] = np.where(near & ((w & F_IP_IN_IP) != 0), o >> 18, 0)
    return out


CHAIN_INLINE = 1 << 31     # ZP_CHAIN_INLINE (offs bit 31, ABI v6)
_RFC_SLOTS = (0, 4, 1, 2, 3, 5)   # HBH, DST1, RT, FRAG, AH, DST2 (slot numbers)


def chain_inline(rec):
    """True where RECORD_DTYPE records carry their outer IPv6 extension chain
    inline (zp_rec_chain_inline, include/zero_packet.h): no ext entry."""
    w = np.asarray(rec["flags"]).astype(np.uint32)
    o = np.asarray(rec["offs"]).astype(np.uint32)
    return (((w >> 26) == 0) & (((w >> 24) & 3) != ETH_CODE_FAR) &
            ((w & (F_EXT | F_IP_IN_IP)) == F_EXT) & ((o & CHAIN_INLINE) != 0))


def inline_chains(rec):
    """zp_rec_chain of every record (EXT_DTYPE [n]; meaningful where
    chain_inline): headers back to back in RFC order, lengths from the
    offs bits 18-29, final_next_header from the L4 reader."""
    rec = np.atleast_1d(rec)
    w = rec["flags"].astype(np.uint32)
    c = rec["offs"].astype(np.uint32) >> 18
    hl = {0: ((c & 7) + 1) * 8, 1: (((c >> 5) & 7) + 1) * 8, 2: np.full_like(c, 8),
          3: (((c >> 8) & 3) + 2) * 4, 4: (((c >> 3) & 3) + 1) * 8,
          5: (((c >> 10) & 3) + 1) * 8}
    out = np.zeros(len(rec), EXT_DTYPE)
    at = np.zeros(len(rec), np.uint32)
    for k in _RFC_SLOTS:
        has = (w & F_EXT_SLOT(k)) != 0
        out["off"][:, k] = np.where(has, at, 0)
        at = at + np.where(has, hl[k], 0)
    out["len"] = at
    out["final_nh"] = np.where(w & F_TCP, 6, np.where(w & F_UDP, 17,
                               np.where(w & F_ICMPV4, 1, 58)))
    return out


def expand_ext(rec, ext):
    """ext (EXT_DTYPE (2, n)) with the entries of inline outer chains rebuilt
    from their records: every entry a record flags is then valid, as the host
    paths (zp_parse_batch_host, zp_parse_one, the ring) deliver them."""
    rec = np.atleast_1d(rec)
    ext = np.array(ext, dtype=EXT_DTYPE).reshape(2, -1)
    m = chain_inline(rec)
    if m.any():
        ext[0][m] = inline_chains(rec[m])
    return ext


def is_far(rec):
    """True where RECORD_DTYPE records hold the far-L4 form."""
    w = np.asarray(rec["flags"]).astype(np.uint32)
    return ((w >> 26) == 0) & (((w >> 24) & 3) == ETH_CODE_FAR)


def _be16(b, i):
    return (b[i] << 8) | b[i + 1]


def _ipv6_chain(frame, ip, chained, x):
    """(extension_headers_len, final_next_header) of the IPv6 header at
    frame[ip:] (ipv6.rs:141, 219-227): from its ext entry x, or its
    next-header byte without a chain."""
    if not chained:
        return 0, frame[ip + 6]
    if x is None:
        # no entry given: the chain is walked again from the frame, as
        # zp_rec_decode does (IPv6Reader::new's extension walk, ipv6.rs:159,
        # through zp_reader_new)
        from . import _lib
        info = np.zeros(1, READER_INFO_DTYPE)
        b = ctypes.create_string_buffer(frame[ip:], max(len(frame) - ip, 1))
        rc = _lib.hip().zp_reader_new(READER_IPV6, ctypes.addressof(b), max(len(frame) - ip, 0),
                                      info.ctypes.data)
        if rc != 0 or not int(info[0]["flags"]) & F_EXT:
            raise ValueError("the record flags an IPv6 extension chain the frame does not hold")
        return int(info[0]["ext"]["len"]), int(info[0]["final_nh"])
    return int(x["len"]), int(x["final_nh"])


def decode(frame, rec, ext=None):
    """One record of `frame` with every field (zp_rec_decode of
    include/zero_packet.h restated): dict flags, err, eth_len, inner_off,
    l4_off, final_nh, inner_final_nh. Both forms; for the far-L4 form the
    Ethernet header length comes from the frame (ethernet.rs:155-179) and
    inner_off follows the outer IP header (IPv4 IHL * 4, ipv4.rs:228-258;
    IPv6 40 + extension_headers_len, ipv6.rs:283-285). ext: the frame's two
    EXT_DTYPE entries where the record flags a chain, or None: the chains are
    then walked again from the frame (zp_reader_new), as in zp_rec_decode."""
    frame = bytes(frame)
    w, o = int(rec["flags"]), int(rec["offs"])
    out = dict(flags=0, err=w >> 26, eth_len=0, inner_off=0, l4_off=0, final_nh=0,
               inner_final_nh=0)
    if out["err"]:
        return out
    flags = w & F_MASK
    out["flags"] = flags
    far = (w >> 24) & 3 == ETH_CODE_FAR
    l4_any = F_TCP | F_UDP | F_ICMPV4 | F_ICMPV6
    if far:
        if not flags & l4_any or not flags & F_IP_IN_IP:
            raise ValueError("far-L4 record without an L4 reader or an ip_in_ip header")
        t = _be16(frame, 12)
        out["eth_len"] = 18 if t == 0x8100 else 22 if t == 0x88A8 else 14
        out["l4_off"] = o
    else:
        out["eth_len"] = 14 + 4 * ((w >> 24) & 3)
        out["l4_off"] = o & L4_NEAR_MAX
        out["inner_off"] = o >> 18 if flags & F_IP_IN_IP else 0
    hl = out["eth_len"]
    chain = 0
    if flags & F_IPV6:
        x = inline_chains(np.array([(w, o)], RECORD_DTYPE))[0] \
            if chain_inline(np.array([(w, o)], RECORD_DTYPE))[0] else (None if ext is None else ext[0])
        chain, out["final_nh"] = _ipv6_chain(frame, hl, flags & F_EXT, x)
    if far:
        out["inner_off"] = hl + 40 + chain if flags & F_IPV6 else hl + (frame[hl] & 15) * 4
    if flags & F_IP_IN_IP_V6:
        out["inner_final_nh"] = _ipv6_chain(frame, out["inner_off"], flags & F_INNER_EXT,
                                            None if ext is None else ext[1])[1]
    return out


def rec_err(rec):
    """err codes of RECORD_DTYPE records (array or scalar)."""
    return np.asarray(rec["flags"]).astype(np.uint32) >> 26


# zp_reader_info (zp_reader_new): Ethernet header_len; IPv6 chain bits,
# final_next_header and offsets.
READER_INFO_DTYPE = np.dtype([("header_len", "<u4"), ("flags", "<u4"), ("final_nh", "u1"),
                              ("reserved", "u1", (3,)), ("ext", EXT_DTYPE)])
assert READER_INFO_DTYPE.itemsize == 28
# zp_reader_kind
(READER_ETHERNET, READER_ARP, READER_IPV4, READER_IPV6, READER_OPTIONS, READER_ROUTING,
 READER_FRAGMENT, READER_AUTH, READER_TCP, READER_UDP, READER_ICMPV4, READER_ICMPV6) = range(12)


def ext_match(got, want, rec):
    """True when the chains the records flag are identical (other entries are
    unspecified by the ABI). got/want: EXT_DTYPE (2, n); rec: RECORD_DTYPE (n,)."""
    mo = (rec["flags"] & F_EXT) != 0
    mi = (rec["flags"] & F_INNER_EXT) != 0
    return (got[0][mo].tobytes() == want[0][mo].tobytes() and
            got[1][mi].tobytes() == want[1][mi].tobytes())


# Presence bits (zero_packet.h ZP_F_*).
F_ETHERNET, F_ARP, F_IPV4, F_IPV6 = 1 << 0, 1 << 1, 1 << 2, 1 << 3
F_IP_IN_IP, F_IP_IN_IP_V6 = 1 << 4, 1 << 5
F_TCP, F_UDP, F_ICMPV4, F_ICMPV6 = 1 << 6, 1 << 7, 1 << 8, 1 << 9
F_EXT, F_INNER_EXT = 1 << 10, 1 << 11
EXT_SLOTS = ["hop_by_hop", "routing", "fragment", "auth_header",
             "destination_1st", "destination_2nd"]


def F_EXT_SLOT(k):
    return 1 << (12 + k)


def F_INNER_EXT_SLOT(k):
    return 1 << (18 + k)


# zp_err codes, in enum order (zero_packet.h).
ERR_NAMES = [
    "OK", "ETH_FRAME_TOO_SHORT", "ETH_SLICE_TOO_SHORT", "ETH_VLAN_TOO_SHORT",
    "ETH_QINQ_TOO_SHORT", "ETH_INVALID_QINQ", "ARP_TOO_SHORT", "ARP_INVALID_OPER",
    "IPV4_TOO_SHORT", "IPV4_VERSION", "IPV4_IHL_TOO_SHORT", "IPV4_HDR_TOO_LONG",
    "IPV4_TOTAL_LENGTH", "IPV4_CHECKSUM", "IPV4_HDR_EXCEEDS", "IPV6_TOO_SHORT",
    "IPV6_VERSION", "EXT_HBH_NOT_FIRST", "EXT_OPTIONS_TOO_SHORT", "EXT_OPTIONS_EXCEEDS",
    "EXT_ROUTING_TOO_SHORT", "EXT_ROUTING_EXCEEDS", "EXT_FRAGMENT_TOO_SHORT",
    "EXT_AUTH_TOO_SHORT", "EXT_AUTH_EXCEEDS", "TCP_TOO_SHORT", "TCP_DATA_OFFSET",
    "TCP_FLAGS", "UDP_TOO_SHORT", "UDP_LENGTH", "ICMP_TOO_SHORT", "ICMPV4_TYPE",
    "ICMPV4_CODE", "ICMPV6_TYPE", "IPV4_L4_CHECKSUM", "IPV6_L4_CHECKSUM",
    "TCP_HDR_EXCEEDS", "OPTIONS_DATA_EXCEEDS",      # reader accessors only (ABI v3)
]
ERR = {name: i for i, name in enumerate(ERR_NAMES)}
