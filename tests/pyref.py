"""Second, independent restatement of PacketParser::parse in pure Python.

Test infrastructure (small inputs only). Used to cross-check the C oracle on
fuzzed / mutated frames; both follow the reference files cited below, written
independently (this one recursive over Python slices with exceptions for
`?`, the C oracle with explicit error returns). Returns the zp_record fields
as a dict so the two can be compared field by field.
"""
from pybuilder import internet_checksum, pseudo_header

ICMPV4_TYPES = {0, 3, 4, 5, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 30, 40, 42, 43, 253, 254}
ICMPV6_TYPES = ({1, 2, 3, 4, 100, 101, 155, 200, 201} | set(range(128, 154)))
SLOTS = ["hop_by_hop", "routing", "fragment", "auth_header", "destination_1st",
         "destination_2nd"]


class Err(Exception):
    def __init__(self, code):
        self.code = code


def be16(b, i):
    return (b[i] << 8) | b[i + 1]


def ext_headers(frame, start, next_header):
    """headers.rs:51-213 -> (dict slot->offset rel. to start, total, final) or None."""
    found = {}
    total = 0
    final = 0
    cur, pos = next_header, start
    while True:
        rem = len(frame) - pos
        if cur == 0:
            if "hop_by_hop" in found:
                break
            if found:
                raise Err("EXT_HBH_NOT_FIRST")
            if rem < 8:
                raise Err("EXT_OPTIONS_TOO_SHORT")
            hl, slot, ex = (frame[pos + 1] + 1) * 8, "hop_by_hop", "EXT_OPTIONS_EXCEEDS"
        elif cur == 43:
            if "routing" in found:
                break
            if rem < 8:
                raise Err("EXT_ROUTING_TOO_SHORT")
            hl, slot, ex = (frame[pos + 1] + 1) * 8, "routing", "EXT_ROUTING_EXCEEDS"
        elif cur == 44:
            if "fragment" in found:
                break
            if rem < 8:
                raise Err("EXT_FRAGMENT_TOO_SHORT")
            hl, slot, ex = 8, "fragment", None
        elif cur == 51:
            if "auth_header" in found:
                break
            if rem < 12:
                raise Err("EXT_AUTH_TOO_SHORT")
            hl, slot, ex = (frame[pos + 1] + 2) * 4, "auth_header", "EXT_AUTH_EXCEEDS"
        elif cur == 60:
            if "destination_2nd" in found:
                break
            if rem < 8:
                raise Err("EXT_OPTIONS_TOO_SHORT")
            hl = (frame[pos + 1] + 1) * 8
            slot = "destination_2nd" if "destination_1st" in found else "destination_1st"
            ex = "EXT_OPTIONS_EXCEEDS"
        else:
            break
        nxt = frame[pos]
        if ex and hl > rem:
            raise Err(ex)
        found[slot] = pos - start
        total += hl
        final = nxt
        cur = nxt
        pos += hl
    if not found:
        return None
    return found, total, final


class State:
    def __init__(self):
        self.f = {}


def parse_ip(frame, pos, v4, level, st):
    """parse_ipv4 / parse_ipv6 (parser.rs:73-107) + parse_protocol (:111-140)."""
    sl = len(frame) - pos
    if v4:
        if sl < 20:
            raise Err("IPV4_TOO_SHORT")
        b0 = frame[pos]
        if b0 >> 4 != 4:
            raise Err("IPV4_VERSION")
        hl = (b0 & 15) * 4
        if hl < 20:
            raise Err("IPV4_IHL_TOO_SHORT")
        if sl < hl:
            raise Err("IPV4_HDR_TOO_LONG")
        if be16(frame, pos + 2) != sl:
            raise Err("IPV4_TOTAL_LENGTH")
        if internet_checksum(frame[pos:pos + hl], 0) != 0:
            raise Err("IPV4_CHECKSUM")
        proto = frame[pos + 9]
        pp = pos + hl
        acc = 0 if proto == 1 else pseudo_header(frame[pos + 12:pos + 16],
                                                 frame[pos + 16:pos + 20], proto, len(frame) - pp)
        csum_err = "IPV4_L4_CHECKSUM"
        ext = None
    else:
        if sl < 40:
            raise Err("IPV6_TOO_SHORT")
        ext = ext_headers(frame, pos + 40, frame[pos + 6])
        if frame[pos] >> 4 != 6:
            raise Err("IPV6_VERSION")
        proto = ext[2] if ext else frame[pos + 6]
        pp = pos + 40 + (ext[1] if ext else 0)
        acc = pseudo_header(frame[pos + 8:pos + 24], frame[pos + 24:pos + 40], proto,
                            len(frame) - pp)
        csum_err = "IPV6_L4_CHECKSUM"
    rem = len(frame) - pp
    l4 = None
    if proto == 6:
        if rem < 20:
            raise Err("TCP_TOO_SHORT")
        if (frame[pp + 12] >> 4) * 4 < 20:
            raise Err("TCP_DATA_OFFSET")
        if frame[pp + 13] == 0:
            raise Err("TCP_FLAGS")
        l4 = "tcp"
    elif proto == 17:
        if rem < 8:
            raise Err("UDP_TOO_SHORT")
        if be16(frame, pp + 4) != rem:
            raise Err("UDP_LENGTH")
        l4 = "udp"
    elif proto == 1:
        if rem < 8:
            raise Err("ICMP_TOO_SHORT")
        if frame[pp] not in ICMPV4_TYPES:
            raise Err("ICMPV4_TYPE")
        if frame[pp + 1] > 15:
            raise Err("ICMPV4_CODE")
        l4 = "icmpv4"
    elif proto == 58:
        if rem < 8:
            raise Err("ICMP_TOO_SHORT")
        if frame[pp] not in ICMPV6_TYPES:
            raise Err("ICMPV6_TYPE")
        l4 = "icmpv6"
    elif proto in (4, 41):
        parse_ip(frame, pp, proto == 4, level + 1, st)
    if l4:
        st.f[l4] = pp
        if internet_checksum(frame[pp:], acc) != 0:
            raise Err(csum_err)
    if level == 0:
        st.f["ipv4" if v4 else "ipv6"] = (pos, ext, proto)
    elif level == 1:
        st.f["ip_in_ip"] = (pos, v4, ext, proto)


def parse(frame):
    """-> dict of zp_record fields (err as name)."""
    frame = bytes(frame)
    st = State()
    try:
        if len(frame) < 64:
            raise Err("ETH_FRAME_TOO_SHORT")
        t = be16(frame, 12)
        hl = 14
        if t == 0x8100:
            hl = 18
        elif t == 0x88A8:
            if be16(frame, 16) != 0x8100:
                raise Err("ETH_INVALID_QINQ")
            hl = 22
        et = be16(frame, hl - 2)
        if et == 0x0806:
            if be16(frame, hl + 6) > 2:
                raise Err("ARP_INVALID_OPER")
            st.f["arp"] = hl
        elif et == 0x0800:
            parse_ip(frame, hl, True, 0, st)
        elif et == 0x86DD:
            parse_ip(frame, hl, False, 0, st)
    except Err as e:
        return {"err": e.code}
    r = {"err": "OK", "flags": {"ethernet"}, "eth_len": hl, "final_nh": 0, "inner_final_nh": 0,
         "inner_off": 0, "l4_off": 0, "ext_len": 0, "ext_off": [0] * 6, "inner_ext_len": 0,
         "inner_ext": [0] * 6}
    f = st.f
    for k in ("arp", "tcp", "udp", "icmpv4", "icmpv6"):
        if k in f:
            r["flags"].add(k)
            if k != "arp":
                r["l4_off"] = f[k]
    if "ipv4" in f:
        r["flags"].add("ipv4")
    if "ipv6" in f:
        r["flags"].add("ipv6")
        _, ext, proto = f["ipv6"]
        r["final_nh"] = proto
        if ext:
            r["flags"].add("ext")
            r["ext_len"] = ext[1]
            for k, name in enumerate(SLOTS):
                if name in ext[0]:
                    r["flags"].add("ext:" + name)
                    r["ext_off"][k] = ext[0][name]
    if "ip_in_ip" in f:
        pos, v4, ext, proto = f["ip_in_ip"]
        r["flags"].add("ip_in_ip")
        r["inner_off"] = pos
        if not v4:
            r["flags"].add("ip_in_ip_v6")
            r["inner_final_nh"] = proto
            if ext:
                r["flags"].add("inner_ext")
                r["inner_ext_len"] = ext[1]
                for k, name in enumerate(SLOTS):
                    if name in ext[0]:
                        r["flags"].add("inner_ext:" + name)
                        r["inner_ext"][k] = ext[0][name]
    return r


FLAG_BITS = {"ethernet": 0, "arp": 1, "ipv4": 2, "ipv6": 3, "ip_in_ip": 4, "ip_in_ip_v6": 5,
             "tcp": 6, "udp": 7, "icmpv4": 8, "icmpv6": 9, "ext": 10, "inner_ext": 11}
for _k, _n in enumerate(SLOTS):
    FLAG_BITS["ext:" + _n] = 12 + _k
    FLAG_BITS["inner_ext:" + _n] = 18 + _k


def to_record_tuple(r, err_codes):
    """dict -> (err, flags, eth_len, final_nh, inner_final_nh, inner_off, l4_off,
    ext_len, ext_off tuple, inner_ext_len, inner_ext tuple) for comparison."""
    if r["err"] != "OK":
        return (err_codes[r["err"]], 0, 0, 0, 0, 0, 0, 0, (0,) * 6, 0, (0,) * 6)
    flags = 0
    for name in r["flags"]:
        flags |= 1 << FLAG_BITS[name]
    return (0, flags, r["eth_len"], r["final_nh"], r["inner_final_nh"], r["inner_off"],
            r["l4_off"], r["ext_len"], tuple(r["ext_off"]), r["inner_ext_len"],
            tuple(r["inner_ext"]))
