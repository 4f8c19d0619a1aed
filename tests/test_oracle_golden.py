"""CPU: pins the oracle (and the test-side builder) to the reference's own
golden vectors and known-answer tests."""
import pytest

import oracle as orc
import pyref
from pybuilder import Builder, internet_checksum

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
]
ERR = {n: i for i, n in enumerate(ERR_NAMES)}


def check_expect(zpkg, frame, rec, ext, expect):
    """Evaluates a fixture's transcribed asserts against a record via the
    PacketParser facade (the same check serves oracle and GPU records)."""
    if "err" in rec.dtype.names:                 # the oracle's unpacked record
        err, rec = int(rec["err"]), orc.pack(rec, ext)[0]
    else:                                        # the ABI's 8-B record
        err = int(rec["flags"]) >> 26
    if not expect["ok"]:
        assert err != 0
        if "err" in expect:
            assert err == ERR[expect["err"]], (ERR_NAMES[err], expect["err"])
        return
    assert err == 0, ERR_NAMES[err]
    p = zpkg.PacketParser.from_record(frame, rec, ext)
    for f in expect.get("some", []):
        assert getattr(p, f) is not None, f
    for f in expect.get("none", []):
        assert getattr(p, f) is None, f
    for key, want in expect.get("fields", {}).items():
        obj, meth = key.split(".")
        got = getattr(getattr(p, obj), meth)()
        if isinstance(got, (bytes, bytearray)):
            got = list(got)
        if isinstance(got, tuple):
            got = [list(x) if isinstance(x, tuple) else x for x in got]
        assert got == want, (key, got, want)
    if "ext_some" in expect:
        eh = p.ipv6.extension_headers
        assert eh is not None
        for slot in expect["ext_some"]:
            assert getattr(eh, slot) is not None, slot
    if "ip_in_ip" in expect:
        assert p.ip_in_ip.kind == expect["ip_in_ip"]


def test_fixture_count(golden):
    # 15 parser.rs packets + 5 builder vectors + 4 builder round trips.
    assert len(golden["fixtures"]) == 24


@pytest.mark.parametrize("idx", range(24))
def test_oracle_matches_reference_asserts(zp, golden, idx):
    fx = golden["fixtures"][idx]
    frame = bytes.fromhex(fx["bytes"])
    err, rec, ext = orc.parse_one(frame)
    assert err == rec["err"]
    check_expect(zp, frame, rec, ext, fx["expect"])


@pytest.mark.parametrize("idx", range(24))
def test_pyref_agrees_with_oracle_on_fixtures(golden, idx):
    frame = bytes.fromhex(golden["fixtures"][idx]["bytes"])
    _, rec, ext = orc.parse_one(frame)
    got = pyref.to_record_tuple(pyref.parse(frame), ERR)
    assert got == orc.record_tuple(rec, ext)


def test_very_complex_packet_structure(golden):
    """builder.rs:1511-1555 plus the offsets that follow from the builder calls:
    QinQ (22) + IPv6 (40) + HBH 16 + Dst1 16 + Rt 16 + Frag 8 + AH 16 + Dst2 16
    -> IPv4 at 150, TCP at 170."""
    fx = [f for f in golden["fixtures"] if f["name"] == "build_parse_very_complex_packet"][0]
    _, rec, ext = orc.parse_one(bytes.fromhex(fx["bytes"]))
    assert rec["err"] == 0
    assert rec["eth_len"] == 22
    assert list(ext[0]["off"]) == [0, 32, 48, 56, 16, 72]   # hbh rt frag ah d1 d2
    assert ext[0]["len"] == 88
    assert rec["final_nh"] == 4 and ext[0]["final_nh"] == 4   # the ABI keeps it in the entry
    assert rec["inner_off"] == 150
    assert rec["l4_off"] == 170


def test_checksum_kats(golden):
    for k in golden["checksum_kats"]:
        assert orc.internet_checksum(k["data"], k["acc"]) == k["checksum"], k["source"]
        assert internet_checksum(k["data"], k["acc"]) == k["checksum"], k["source"]
    p = golden["pseudo_header_kat"]
    assert orc.pseudo_header(p["src"], p["dst"], p["protocol"], p["length"]) == p["sum"]


def test_pybuilder_reproduces_reference_vectors(golden):
    """The test-side builder restatement must emit the builder's exact bytes."""
    vec = {v["name"]: bytes.fromhex(v["bytes"]) for v in golden["builder_vectors"]}
    m1 = [0x34, 0x97, 0xf6, 0x94, 0x02, 0x0f]
    m2 = [0x04, 0xb4, 0xfe, 0x9a, 0x81, 0xc7]
    ip1, ip2 = [192, 168, 1, 1], [192, 168, 1, 2]
    bcast = [0xff] * 6
    b = Builder(42).ethernet(m1, bcast, 2054).arp(1, 2048, 6, 4, 1, m1, ip1, [0] * 6, ip2)
    assert b.build() == vec["arp_in_ethernet"]
    b = (Builder(54).ethernet(m1, m2, 2048)
         .ipv4(99, 5, 99, 123, 12345, 54321, 99, 12345, 123, 6, ip1, ip2)
         .tcp(ip1, 99, ip2, 11, 123, 321, 11, 99, 99, 4321, 1234))
    assert b.build() == vec["tcp_in_ipv4_in_ethernet"]
    b = (Builder(54).ethernet(m1, m2, 2048)
         .ipv4(99, 5, 99, 123, 12345, 54321, 99, 12345, 123, 6, ip1, ip2)
         .udp(ip1, 99, ip2, 11, 4321))
    assert b.build() == vec["udp_in_ipv4_in_ethernet"]
    b = (Builder(64).ethernet(m1, m2, 2048)
         .ipv4(4, 5, 99, 123, 12345, 54321, 99, 12345, 123, 1, ip1, ip2).icmpv4(8, 0))
    assert b.build() == vec["icmpv4_in_ipv4_in_ethernet"]
    s6 = [0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0, 0, 0, 0, 0x8a, 0x2e, 0x03, 0x70, 0x73, 0x34]
    d6 = [0xfe, 0x80, 0, 0, 0, 0, 0, 0, 0x02, 0x02, 0xb3, 0xff, 0xfe, 0x1e, 0x83, 0x29]
    b = (Builder(64).ethernet(m1, m2, 34525).ipv6(6, 5, 4, 31, 17, 10, s6, d6)
         .udp(s6, 99, d6, 80, 10))
    assert b.build() == vec["build_parse_ipv6"]
