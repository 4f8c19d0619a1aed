"""Debug formatting of parsed packets (CPU only).

Parity unpinned: the reference's tests assert no Debug output, and the Rust
reference cannot be run here. The expected strings below follow the Debug
impls cited in zero-packet_amd/debugfmt.py with Rust's debug_struct /
debug_tuple / slice rules.
"""
import re

import oracle as orc

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
    err, rec, ext = orc.parse_one(frame)
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
        err, rec, ext = orc.parse_one(frame)
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
