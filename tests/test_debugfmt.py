"""Debug formatting of parsed packets (CPU only).

The reference's tests assert no Debug output and the Rust reference cannot
run here, so no output string is pinned. What is pinned is the shape: the
golden file's `debug_impls` (extracted by tests/golden/make_golden.py from
the reference's `impl fmt::Debug` blocks, the derived Debug types and the
misc.rs helpers) gives every struct name, field name, field order and what
each field prints (getter + its return type, member, MAC / IPv6 string,
IpFormatter). test_debug_follows_the_reference_impls rebuilds the expected
`{:?}` text from that data and the getters (themselves pinned by the
reference's getter tests) with Rust's std rules for debug_struct, Option,
tuple variants, slices, integers, bools and &str, and compares it with the
facade's output for every reader the fixtures hold and every parsed golden
packet. The hand-written strings below are kept as readable examples.
"""
import re

import pytest

import oracle as orc
from test_getters import READER_CLS, built

IPV6_UDP = ('PacketParser { ethernet: Some(EthernetFrame { dest_mac: "04:b4:fe:9a:81:c7", '
            'src_mac: "34:97:f6:94:02:0f", ethertype: 34525 }), arp: None, ipv4: None, '
            'ipv6: Some(IPv6Packet { version: 6, traffic_class: 5, flow_label: 4, '
            'payload_length: 31, next_header: 17, hop_limit: 10, '
            'src_addr: "2001:0db8:85a3:0000:0000:8a2e:0370:7334", '
            'dest_addr: "fe80:0000:0000:0000:0202:b3ff:fe1e:8329", extension_headers: None, '
            'extension_headers_len: 0 }), ip_in_ip: None, tcp: None, '
            'udp: Some(UdpDatagram { src_port: 99, dest_port: 80, length: 10 }), '
            'icmpv4: None, icmpv6: None }')

PRETTY_UDP = """UdpDatagram {
    src_port: 99,
    dest_port: 80,
    length: 10,
}"""


def parsed(zp, golden, name):
    fx = next(f for f in golden["fixtures"] if f["name"] == name)
    frame = bytes.fromhex(fx["bytes"])
    err, rec, ext = orc.parse_one_abi(frame)
    assert err == 0
    return zp.PacketParser.from_record(frame, rec, ext)


def test_debug_compact(zp, golden):
    p = parsed(zp, golden, "build_parse_ipv6")
    assert p.debug() == IPV6_UDP
    assert zp.debugfmt.debug(p.udp, pretty=True) == PRETTY_UDP


def test_debug_complex_packet(zp, golden):
    p = parsed(zp, golden, "build_parse_very_complex_packet")
    s = p.debug()
    assert "ip_in_ip: Some(Ipv4(IPv4Packet { version: 4, ihl: 5," in s
    assert "src_ip: 192.168.1.1, dest_ip: 192.168.1.2 }))" in s
    assert "fragment: Some(FragmentHeader { next_header: 51, reserved: 0, fragment_offset: 255, " \
           "res: 0, m_flag: true, identification: 67438087 })" in s
    assert "total_headers_len: 88, final_next_header: 4 }), extension_headers_len: 88 })" in s


def test_debug_pretty_matches_compact(zp, golden):
    """{:#?} is {:?} with line breaks, indentation and trailing commas."""
    n = 0
    for fx in golden["fixtures"]:
        frame = bytes.fromhex(fx["bytes"])
        err, rec, ext = orc.parse_one_abi(frame)
        if err:
            continue
        p = zp.PacketParser.from_record(frame, rec, ext)
        compact, pretty = p.debug(), p.debug(pretty=True)
        squash = re.sub(r",\n\s*([\]\)}])", r"\1", pretty)
        squash = re.sub(r"\(\n\s*", "(", squash)
        squash = re.sub(r"\[\n\s*", "[", squash)
        squash = re.sub(r"\{\n\s*", "{ ", squash)
        squash = re.sub(r",\n\s*", ", ", squash)
        squash = squash.replace("}", " }").replace("  }", " }")
        assert squash.replace(" ", "") == compact.replace(" ", ""), fx["name"]
        n += 1
    assert n >= 8


# ---- the reference's Debug impls as data -----------------------------------

def _rust(v, ty):
    """Rust std Debug of a getter value of reference return type `ty`."""
    if ty.startswith("Result<"):
        return v if isinstance(v, str) else f"Ok({_rust(v, '&[u8]')})"
    if ty == "bool":
        return "true" if v else "false"
    if ty == "&[u8]":
        return "[" + ", ".join(str(int(x)) for x in v) + "]"
    assert ty in ("u8", "u16", "u32", "usize"), ty
    return str(int(v))


def _expect(zp, node, D):
    """Expected {:?} of a facade value, from the reference's Debug data."""
    P = zp.parser
    h = D["helpers"]
    hexc = h["hex_chars"][0]
    if node is None:
        return "None"
    if isinstance(node, P.PacketParser):
        items = D["PacketParser"]["items"]
        return "PacketParser { " + ", ".join(
            f"{k}: " + ("None" if getattr(node, k) is None
                        else f"Some({_expect(zp, getattr(node, k), D)})") for k in items) + " }"
    if isinstance(node, P.IpInIp):
        v4, v6 = D["IpInIp"]["items"]
        return f"{v4 if node.kind == 'ipv4' else v6}({_expect(zp, node.reader, D)})"
    if isinstance(node, P.ExtensionHeaders):
        parts = []
        for k in D["ExtensionHeaders"]["items"]:
            v = getattr(node, k)
            if k in ("total_headers_len", "final_next_header"):
                parts.append(f"{k}: {int(v)}")
            else:
                parts.append(f"{k}: " + ("None" if v is None else f"Some({_expect(zp, v, D)})"))
        return "ExtensionHeaders { " + ", ".join(parts) + " }"
    impl = D["impls"][type(node).__name__]
    parts = []
    for key, kind, src, *ret in impl["fields"]:
        if kind == "getter":
            try:
                v = getattr(node, src)()
            except P.ZeroPacketError as e:
                assert ret[0].startswith("Result<")
                v = f'Err("{e}")'
            val = _rust(v, ret[0])
        elif kind == "member":
            v = getattr(node, src)
            if src == "extension_headers":
                val = "None" if v is None else f"Some({_expect(zp, v, D)})"
            else:
                val = str(int(v))
        elif kind == "mac":
            b = getattr(node, src)()
            assert h["mac_separator_every"] == 1
            val = '"' + ":".join(hexc[x >> 4] + hexc[x & 15] for x in b) + '"'
        elif kind == "ipv6":
            b = getattr(node, src)()
            g = h["ipv6_separator_every"]
            val = '"' + ":".join("".join(hexc[x >> 4] + hexc[x & 15] for x in b[i:i + g])
                                 for i in range(0, len(b), g)) + '"'
        else:
            assert kind == "ipv4"
            b = getattr(node, src)()
            val = h["ipv4_format"].replace("{}", "%d") % tuple(b[:4])
        parts.append(f"{key}: {val}")
    return impl["struct"] + " { " + ", ".join(parts) + " }"


def test_debug_impls_fixture(golden):
    D = golden["debug_impls"]
    assert sorted(D["impls"]) == sorted(READER_CLS.values())
    assert D["impls"]["TcpReader"]["fields"][3][:3] == ["acknowledgment_number", "getter",
                                                          "ack_number"]
    assert D["impls"]["Icmpv4Reader"]["fields"][0][0] == "type"
    assert D["PacketParser"]["items"][4] == "ip_in_ip" and D["IpInIp"]["items"] == ["Ipv4", "Ipv6"]
    assert D["helpers"]["hex_chars"] == ["0123456789abcdef"] * 2


def test_debug_follows_the_reference_impls(zp, golden):
    D = golden["debug_impls"]
    seen = set()
    # every reader of the reference's getter tests, built with their values
    for g, frame, at, *_ in built(zp, golden):
        r = getattr(zp, READER_CLS[g["reader"]]).new(frame[at:])
        assert zp.debugfmt.debug(r) == _expect(zp, r, D), g["reader"]
        seen.add(type(r).__name__)
    # every golden packet that parses, whole
    n = 0
    for fx in golden["fixtures"]:
        frame = bytes.fromhex(fx["bytes"])
        err, rec, ext = orc.parse_one_abi(frame)
        if err:
            continue
        p = zp.PacketParser.from_record(frame, rec, ext)
        assert p.debug() == _expect(zp, p, D), fx["name"]
        n += 1
    assert n >= 8 and seen == set(READER_CLS.values())


@pytest.mark.gpu
def test_debug_of_gpu_records(zp, golden):
    """Row f4 through the product path: the golden packets, 2,048 c5 frames,
    512 c4 frames (extension chains) and the far-L4 frames parsed ON THE GPU,
    through the device batch (zp_parse_batch_device) and through
    PacketParser.parse (zp_parse_one). Their {:?} and {:#?} text equals the
    text of the oracle's records and the text the reference's Debug impls
    give (misc.rs:243-290, ipv4.rs:267-287, ...)."""
    import numpy as np
    import torch
    from test_l4_far import CASES, deep_frame
    D = golden["debug_impls"]
    frames = [bytes.fromhex(fx["bytes"]) for fx in golden["fixtures"]]
    for cfg, n in (("c5", 2048), ("c4", 512)):
        a, o, l = zp.batch.generate_host(cfg, n, first=777)
        frames += [a[int(o[i]):int(o[i]) + int(l[i])].tobytes() for i in range(n)]
    frames += [deep_frame(lv, **kw)[0] for lv, kw in CASES]
    offs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.int64)
    arena = np.frombuffer(b"".join(frames) + bytes(64), np.uint8).copy()
    lens = np.array([len(f) for f in frames], np.int32)
    d = torch.device("cuda:0")
    r, e = zp.batch.parse_batch(torch.from_numpy(arena).to(d), torch.from_numpy(offs).to(d),
                                torch.from_numpy(lens).to(d))
    got, gext = zp.batch.records_to_numpy(r, e)
    ok = 0
    for k, f in enumerate(frames):
        err, rec, ext = orc.parse_one_abi(f)
        assert int(got[k]["flags"]) >> 26 == err
        if err:
            continue
        want = zp.PacketParser.from_record(f, rec, ext)
        batch = zp.PacketParser.from_record(f, got[k], gext[:, k])
        one = zp.PacketParser.parse(f)
        text = want.debug()
        assert text == _expect(zp, want, D)
        assert batch.debug() == text and one.debug() == text, k
        pretty = want.debug(pretty=True)
        assert batch.debug(pretty=True) == pretty and one.debug(pretty=True) == pretty, k
        ok += 1
    assert ok >= 2560
