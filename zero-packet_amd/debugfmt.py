"""`{:?}` / `{:#?}` formatting of parsed packets, as the reference prints them
(SURVEY.md §8(f) row 4).

Follows the reference's Debug impls field by field: EthernetReader
(ethernet.rs:265-279, MACs via bytes_to_mac misc.rs:243-261), ArpReader
(arp.rs:229-250), IPv4Reader (ipv4.rs:267-287, IpFormatter misc.rs:282-290),
IPv6Reader (ipv6.rs:288-309, bytes_to_ipv6 misc.rs:263-280), the extension
readers (options.rs:156-164, routing.rs:197-208, fragment.rs:175-187,
authentication.rs:202-213), TcpReader (tcp.rs:246-261), UdpReader
(udp.rs:156-164), Icmpv4Reader (icmpv4.rs:137-145), Icmpv6Reader
(icmpv6.rs:134-142), and the derived Debug of PacketParser (parser.rs:21-32),
IpInIp (misc.rs:5-9) and ExtensionHeaders (headers.rs:18-28), rendered with
Rust's debug_struct / debug_tuple / slice rules (compact, and `{:#?}` with
4-space indentation and trailing commas).
"""
from . import parser as P


class _Struct:
    def __init__(self, name, fields):
        self.name, self.fields = name, fields


class _Tuple:
    def __init__(self, name, items):
        self.name, self.items = name, items


class _List:
    def __init__(self, items):
        self.items = items


class _Raw:
    def __init__(self, text):
        self.text = text


def _str(s):
    """Debug of &str: quoted (the formatted MAC / IPv6 strings need no escapes)."""
    return _Raw('"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"')


def _num(v):
    return _Raw(str(int(v)))


def _bool(v):
    return _Raw("true" if v else "false")


def _opt(node):
    return _Raw("None") if node is None else _Tuple("Some", [node])


def _indent(text):
    return "\n".join("    " + line if line else line for line in text.split("\n"))


def render(node, pretty=False):
    if isinstance(node, _Raw):
        return node.text
    if isinstance(node, _Tuple):
        if pretty:
            inner = "".join(_indent(render(x, True)) + ",\n" for x in node.items)
            return f"{node.name}(\n{inner})"
        return f"{node.name}(" + ", ".join(render(x) for x in node.items) + ")"
    if isinstance(node, _List):
        if not node.items:
            return "[]"
        if pretty:
            return "[\n" + "".join(_indent(render(x, True)) + ",\n" for x in node.items) + "]"
        return "[" + ", ".join(render(x) for x in node.items) + "]"
    if isinstance(node, _Struct):
        if not node.fields:
            return node.name
        if pretty:
            body = "".join(_indent(f"{k}: {render(v, True)}") + ",\n" for k, v in node.fields)
            return f"{node.name} {{\n{body}}}"
        return f"{node.name} {{ " + ", ".join(f"{k}: {render(v)}" for k, v in node.fields) + " }"
    raise TypeError(node)


def _mac(b):                       # bytes_to_mac (misc.rs:243-261)
    return ":".join(f"{x:02x}" for x in b)


def _ipv6(b):                      # bytes_to_ipv6 (misc.rs:263-280): 2 bytes per group
    return ":".join(f"{b[k]:02x}{b[k + 1]:02x}" for k in range(0, 16, 2))


def _ipv4(b):                      # IpFormatter (misc.rs:282-290): unquoted
    return _Raw(f"{b[0]}.{b[1]}.{b[2]}.{b[3]}")


def _bytes(b):
    return _List([_num(x) for x in b])


def _result(fn):
    try:
        return _Tuple("Ok", [_bytes(fn())])
    except P.ZeroPacketError as e:
        return _Tuple("Err", [_str(str(e))])


def node_of(r):
    """Debug tree of one reader / parser value."""
    if r is None:
        return _Raw("None")
    if isinstance(r, P.EthernetReader):
        return _Struct("EthernetFrame", [("dest_mac", _str(_mac(r.dest_mac()))),
                                         ("src_mac", _str(_mac(r.src_mac()))),
                                         ("ethertype", _num(r.ethertype()))])
    if isinstance(r, P.ArpReader):
        return _Struct("Arp", [
            ("hardware_type", _num(r.htype())), ("protocol_type", _num(r.ptype())),
            ("hardware_address_length", _num(r.hlen())),
            ("protocol_address_length", _num(r.plen())), ("operation", _num(r.oper())),
            ("sender_hardware_address", _str(_mac(r.sha()))),
            ("sender_protocol_address", _ipv4(r.spa())),
            ("target_hardware_address", _str(_mac(r.tha()))),
            ("target_protocol_address", _ipv4(r.tpa()))])
    if isinstance(r, P.IPv4Reader):
        return _Struct("IPv4Packet", [
            ("version", _num(r.version())), ("ihl", _num(r.ihl())), ("dscp", _num(r.dscp())),
            ("ecn", _num(r.ecn())), ("total_length", _num(r.total_length())),
            ("identification", _num(r.id())), ("flags", _num(r.flags())),
            ("fragment_offset", _num(r.fragment_offset())), ("ttl", _num(r.ttl())),
            ("protocol", _num(r.protocol())), ("checksum", _num(r.checksum())),
            ("src_ip", _ipv4(r.src_ip())), ("dest_ip", _ipv4(r.dest_ip()))])
    if isinstance(r, P.IPv6Reader):
        return _Struct("IPv6Packet", [
            ("version", _num(r.version())), ("traffic_class", _num(r.traffic_class())),
            ("flow_label", _num(r.flow_label())), ("payload_length", _num(r.payload_length())),
            ("next_header", _num(r.next_header())), ("hop_limit", _num(r.hop_limit())),
            ("src_addr", _str(_ipv6(r.src_addr()))), ("dest_addr", _str(_ipv6(r.dest_addr()))),
            ("extension_headers", _opt(None if r.extension_headers is None
                                       else node_of(r.extension_headers))),
            ("extension_headers_len", _num(r.extension_headers_len))])
    if isinstance(r, P.ExtensionHeaders):
        return _Struct("ExtensionHeaders", [
            ("hop_by_hop", _opt(r.hop_by_hop and node_of(r.hop_by_hop))),
            ("routing", _opt(r.routing and node_of(r.routing))),
            ("fragment", _opt(r.fragment and node_of(r.fragment))),
            ("auth_header", _opt(r.auth_header and node_of(r.auth_header))),
            ("destination_1st", _opt(r.destination_1st and node_of(r.destination_1st))),
            ("destination_2nd", _opt(r.destination_2nd and node_of(r.destination_2nd))),
            ("total_headers_len", _num(r.total_headers_len)),
            ("final_next_header", _num(r.final_next_header))])
    if isinstance(r, P.OptionsHeaderReader):
        return _Struct("OptionsHeaderReader", [
            ("next_header", _num(r.next_header())), ("header_ext_len", _num(r.header_ext_len())),
            ("options", _result(r.options))])
    if isinstance(r, P.RoutingHeaderReader):
        return _Struct("RoutingExtensionHeader", [
            ("next_header", _num(r.next_header())), ("header_ext_len", _num(r.header_ext_len())),
            ("routing_type", _num(r.routing_type())), ("segments_left", _num(r.segments_left())),
            ("data", _bytes(r.data()))])
    if isinstance(r, P.FragmentHeaderReader):
        return _Struct("FragmentHeader", [
            ("next_header", _num(r.next_header())), ("reserved", _num(r.reserved())),
            ("fragment_offset", _num(r.fragment_offset())), ("res", _num(r.res())),
            ("m_flag", _bool(r.m_flag())), ("identification", _num(r.identification()))])
    if isinstance(r, P.AuthenticationHeaderReader):
        if r.header_len() < 12 <= len(r.bytes):
            # &bytes[12..header_len] with header_len < 12: the reference panics
            raise RuntimeError("AuthenticationHeaderReader Debug: slice index starts at 12 "
                               f"but ends at {r.header_len()} (the reference panics)")
        return _Struct("AuthenticationHeader", [
            ("next_header", _num(r.next_header())), ("payload_len", _num(r.payload_len())),
            ("reserved", _num(r.reserved())), ("spi", _num(r.spi())),
            ("sequence_number", _num(r.sequence_number())),
            ("authentication_data", _result(r.authentication_data))])
    if isinstance(r, P.TcpReader):
        return _Struct("TcpSegment", [
            ("src_port", _num(r.src_port())), ("dest_port", _num(r.dest_port())),
            ("sequence_number", _num(r.sequence_number())),
            ("acknowledgment_number", _num(r.ack_number())),
            ("data_offset", _num(r.data_offset())), ("reserved", _num(r.reserved())),
            ("flags", _num(r.flags())), ("window_size", _num(r.window_size())),
            ("checksum", _num(r.checksum())), ("urgent_pointer", _num(r.urgent_pointer()))])
    if isinstance(r, P.UdpReader):
        return _Struct("UdpDatagram", [("src_port", _num(r.src_port())),
                                       ("dest_port", _num(r.dest_port())),
                                       ("length", _num(r.length()))])
    if isinstance(r, P.Icmpv4Reader):
        return _Struct("Icmpv4Packet", [("type", _num(r.icmp_type())),
                                        ("code", _num(r.icmp_code())),
                                        ("checksum", _num(r.checksum()))])
    if isinstance(r, P.Icmpv6Reader):
        return _Struct("Icmpv6Packet", [("icmp_type", _num(r.icmp_type())),
                                        ("icmp_code", _num(r.icmp_code())),
                                        ("checksum", _num(r.checksum()))])
    if isinstance(r, P.IpInIp):
        return _Tuple("Ipv4" if r.kind == "ipv4" else "Ipv6", [node_of(r.reader)])
    if isinstance(r, P.PacketParser):
        return _Struct("PacketParser", [(f, _opt(None if getattr(r, f) is None
                                                 else node_of(getattr(r, f))))
                                        for f in P.PacketParser.FIELDS])
    raise TypeError(f"no Debug for {type(r).__name__}")


def debug(value, pretty=False):
    """format!("{:?}", value) (pretty: "{:#?}")."""
    return render(node_of(value), pretty)
