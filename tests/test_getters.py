"""The reference's per-reader `getters_and_setters` tests as fixtures
(tests/golden/parse_golden.json "reader_getters", transcribed from
ethernet.rs:285-310, arp.rs:257-289, ipv4.rs:293-346, ipv6.rs:315-361,
options.rs:170-194, routing.rs:213-240, fragment.rs:192-226,
authentication.rs:219-250, tcp.rs:268-317, udp.rs:171-202, icmpv4.rs:151-174,
icmpv6.rs:149-187 by tests/golden/make_golden.py).

Each test's header is built with the same field values by the oracle's
builder restatement (zpo_build, pinned by the reference's builder vectors),
in a buffer of the test's size. Then:
  CPU  the Python facade's checked constructor + getters return the values
       the reference test asserts, and so do the oracle's column getters
       (zpo_columns) over a record that points at the header;
  GPU  the column kernel (zp_extract_columns_device) returns them too.
This pins the bit positions of the getters (e.g. the fragment offset split,
fragment.rs:125-127, the IPv6 traffic class / flow label) on the reference's
own values rather than on a restatement alone.
"""
import numpy as np
import pytest

import oracle as orc

M = [0x02, 0, 0, 0, 0, 0x01]
IP4 = [10, 0, 0, 1]
IP6 = [0xfe, 0x80] + [0] * 13 + [1]


def _fx(golden):
    return {g["reader"]: g for g in golden["reader_getters"]}


def _sets(g):
    return {k: v for k, v in g["sets"]}


def chain_for(zp, g):
    """(chain, buffer length, header offset, record flags, l4 offset, final_nh)
    building the fixture's header with its values. Fields the builder has no
    slot for (fragment reserved/res, auth reserved) keep the zero buffer's
    bytes, which is what the fixture sets them to (asserted)."""
    C, B = zp.builder.Chain, zp.builder
    s, r = _sets(g), g["reader"]
    n = g["buffer_len"]
    F = zp.records
    eth4 = lambda c, proto: c.ethernet(M, M, 0x0800).ipv4(4, 5, 0, 0, 20 + n, 0, 0, 0, 64, proto,
                                                            IP4, IP4)
    eth6 = lambda c, nh: c.ethernet(M, M, 0x86DD).ipv6(6, 0, 0, n, nh, 64, IP6, IP6)
    if r == "ethernet":
        return C().ethernet(s["src_mac"], s["dest_mac"], s["ethertype"]), n, 0, F.F_ETHERNET, 0, 0
    if r == "arp":
        c = C().ethernet(M, M, 0x0806).arp(s["htype"], s["ptype"], s["hlen"], s["plen"], s["oper"],
                                           s["sha"], s["spa"], s["tha"], s["tpa"])
        return c, 14 + n, 14, F.F_ETHERNET | F.F_ARP, 0, 0
    if r == "ipv4":
        assert s["checksum"] is None                       # set_checksum(): computed
        c = C().ethernet(M, M, 0x0800).ipv4(s["version"], s["ihl"], s["dscp"], s["ecn"],
                                            s["total_length"], s["id"], s["flags"],
                                            s["fragment_offset"], s["ttl"], s["protocol"],
                                            s["src_ip"], s["dest_ip"])
        return c, 14 + n, 14, F.F_ETHERNET | F.F_IPV4, 0, 0
    if r == "ipv6":
        c = C().ethernet(M, M, 0x86DD).ipv6(s["version"], s["traffic_class"], s["flow_label"],
                                            s["payload_length"], s["next_header"], s["hop_limit"],
                                            s["src_addr"], s["dest_addr"])
        return c, 14 + n, 14, F.F_ETHERNET | F.F_IPV6, 0, s["next_header"]
    if r == "options":
        c = eth6(C(), 0).hop_by_hop(s["next_header"], s["header_ext_len"], s["options"])
        return c, 54 + n, 54, 0, 0, 0
    if r == "routing":
        c = eth6(C(), 43).routing_header(s["next_header"], s["header_ext_len"], s["routing_type"],
                                         s["segments_left"], s["data"])
        return c, 54 + n, 54, 0, 0, 0
    if r == "fragment":
        assert s["reserved"] == 0 and s["res"] == 0        # zero-buffer bytes
        c = eth6(C(), 44).fragment_header(s["next_header"], s["fragment_offset"], s["m_flag"],
                                          s["identification"])
        return c, 54 + n, 54, 0, 0, 0
    if r == "authentication":
        assert s["reserved"] == 0
        c = eth6(C(), 51).authentication_header(s["next_header"], s["payload_len"], s["spi"],
                                                s["sequence_number"], s["authentication_data"])
        return c, 54 + n, 54, 0, 0, 0
    if r == "tcp":
        c = eth4(C(), 6).tcp(IP4, s["src_port"], IP4, s["dest_port"], s["sequence_number"],
                             s["ack_number"], s["data_offset"], s["reserved"], s["flags"],
                             s["window_size"], s["urgent_pointer"])
        return c, 34 + n, 34, F.F_ETHERNET | F.F_IPV4 | F.F_TCP, 34, 0
    if r == "udp":
        c = eth4(C(), 17).udp(IP4, s["src_port"], IP4, s["dest_port"], s["length"])
        return c, 34 + n, 34, F.F_ETHERNET | F.F_IPV4 | F.F_UDP, 34, 0
    if r == "icmpv4":
        c = eth4(C(), 1).icmpv4(s["icmp_type"], s["icmp_code"])
        return c, 34 + n, 34, F.F_ETHERNET | F.F_IPV4 | F.F_ICMPV4, 34, 0
    if r == "icmpv6":
        c = eth6(C(), 58).icmpv6(IP6, IP6, s["icmp_type"], s["icmp_code"])
        return c, 54 + n, 54, F.F_ETHERNET | F.F_IPV6 | F.F_ICMPV6, 54, 58
    raise KeyError(r)


READER_CLS = {"ethernet": "EthernetReader", "arp": "ArpReader", "ipv4": "IPv4Reader",
              "ipv6": "IPv6Reader", "options": "OptionsHeaderReader",
              "routing": "RoutingHeaderReader", "fragment": "FragmentHeaderReader",
              "authentication": "AuthenticationHeaderReader", "tcp": "TcpReader",
              "udp": "UdpReader", "icmpv4": "Icmpv4Reader", "icmpv6": "Icmpv6Reader"}


def built(zp, golden):
    """Every fixture's frame built by the oracle builder: [(fixture, frame,
    header offset, flags, l4 offset, final_nh)]."""
    out = []
    for g in golden["reader_getters"]:
        c, size, at, flags, l4, fnh = chain_for(zp, g)
        b = zp.builder.BuildBatch().add(c)
        ops, op_start, data = b.pack()
        arena = np.zeros(size + 64, np.uint8)
        res = orc.build_batch(arena, np.array([0], np.uint64), np.array([size], np.uint32), ops,
                              op_start, data).view(zp.builder.RESULT_DTYPE)[0]
        assert res["err"] == 0, (g["reader"], int(res["err"]))
        out.append((g, arena[:size].tobytes(), at, flags, l4, fnh))
    return out


def _norm(v):
    if isinstance(v, (bytes, bytearray)):
        return list(v)
    return v


def test_fixtures_cover_the_twelve_readers(golden):
    fx = _fx(golden)
    assert sorted(fx) == sorted(READER_CLS)
    for g in fx.values():
        assert g["asserts"] and g["buffer_len"], g["reader"]
    # the values the round-2 verdict names: TCP seq/ack/window, IPv6 traffic
    # class / flow label, the fragment offset
    assert dict(fx["tcp"]["asserts"])["window_size"] == 1024
    assert dict(fx["ipv6"]["asserts"])["flow_label"] == 4
    assert dict(fx["fragment"]["asserts"])["fragment_offset"] == 255


def test_facade_getters_return_the_reference_values(zp, golden):
    for g, frame, at, *_ in built(zp, golden):
        r = getattr(zp, READER_CLS[g["reader"]]).new(frame[at:])
        for getter, want in g["asserts"]:
            assert _norm(getattr(r, getter)()) == want, (g["reader"], getter)


# zp_col -> (fixture reader, value from the fixture's asserts)
def column_expect(g, at, l4):
    a = dict(g["asserts"])
    r = g["reader"]
    if r == "ethernet":
        return {"src_mac": a["src_mac"], "dest_mac": a["dest_mac"], "ethertype": a["ethertype"]}
    if r == "arp":
        return {"arp_oper": a["oper"]}
    if r == "ipv4":
        return {"ip_version": a["version"], "protocol": a["protocol"], "ttl": a["ttl"],
                "tos": (a["dscp"] << 2) | a["ecn"], "ip_id": a["id"], "ip_len": a["total_length"],
                "src_addr": a["src_ip"] + [0] * 12, "dest_addr": a["dest_ip"] + [0] * 12}
    if r == "ipv6":
        return {"ip_version": a["version"], "tos": a["traffic_class"], "ip_id": a["flow_label"],
                "ip_len": a["payload_length"], "protocol": a["next_header"],
                "ttl": a["hop_limit"], "src_addr": a["src_addr"], "dest_addr": a["dest_addr"]}
    if r == "tcp":
        return {"l4_proto": 6, "src_port": a["src_port"], "dest_port": a["dest_port"],
                "tcp_seq": a["sequence_number"], "tcp_ack": a["ack_number"],
                "tcp_flags": a["flags"], "tcp_window": a["window_size"],
                "payload_off": l4 + 4 * a["data_offset"]}
    if r == "udp":
        return {"l4_proto": 17, "src_port": a["src_port"], "dest_port": a["dest_port"],
                "payload_off": l4 + 8}
    if r in ("icmpv4", "icmpv6"):
        return {"l4_proto": 1 if r == "icmpv4" else 58, "icmp_type": a["icmp_type"],
                "icmp_code": a["icmp_code"]}
    return {}


def _records(zp, frames):
    """Frames packed + one record per frame pointing at its fixture header."""
    rec = np.zeros(len(frames), orc.RECORD_DTYPE)       # unpacked; orc.pack for the ABI
    offs, pos = [], 0
    for i, (g, frame, at, flags, l4, fnh) in enumerate(frames):
        offs.append(pos)
        pos += len(frame)
        rec[i]["flags"] = flags
        rec[i]["eth_len"] = 14
        rec[i]["l4_off"] = l4
        rec[i]["final_nh"] = fnh
    arena = np.frombuffer(b"".join(f for _, f, *_ in frames) + bytes(64), np.uint8).copy()
    return arena, np.array(offs, np.uint64), np.array([len(f) for _, f, *_ in frames], np.uint32), rec


def _check_columns(frames, cols, get):
    checked = 0
    for i, (g, frame, at, flags, l4, fnh) in enumerate(frames):
        for name, want in column_expect(g, at, l4).items():
            got = get(cols[name], i)
            assert got == want, (g["reader"], name, got, want)
            checked += 1
    return checked


def test_oracle_columns_return_the_reference_values(zp, golden):
    frames = [f for f in built(zp, golden) if f[3]]
    arena, offs, lens, rec = _records(zp, frames)
    cols = orc.columns(arena, offs, lens, rec)
    get = lambda c, i: c[i].tolist() if c.ndim > 1 else int(c[i])
    assert _check_columns(frames, cols, get) == 38


@pytest.mark.gpu
def test_gpu_columns_return_the_reference_values(zp, golden):
    import torch
    d = torch.device("cuda:0")
    frames = [f for f in built(zp, golden) if f[3]]
    arena, offs, lens, rec = _records(zp, frames)
    cols = zp.columns.extract(torch.from_numpy(arena).to(d),
                              torch.from_numpy(offs.astype(np.int64)).to(d),
                              torch.from_numpy(lens.astype(np.int32)).to(d),
                              torch.from_numpy(orc.pack(rec, np.zeros((2, len(rec)), orc.EXT_DTYPE)).view(np.uint8).reshape(-1, 8)).to(d))
    cols = {k: v.cpu().numpy() for k, v in cols.items()}
    get = lambda c, i: c[i].tolist() if c.ndim > 1 else int(c[i])
    assert _check_columns(frames, cols, get) == 38
