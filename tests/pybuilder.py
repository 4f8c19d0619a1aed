"""Test-side restatement of the reference PacketBuilder writers (builder.rs).

The builder is outside the hot path; tests use this
restatement to construct frames for the reference's build->parse round-trip
tests and for edge cases. It follows the writers field by field, including
their u8 truncation quirks (e.g. `version << 4` in ipv4.rs:37), and it is
pinned by reproducing the builder's exact `should_be` vectors
(builder.rs:1052-1055, 1097-1101, 1161-1165, 1212-1216, 1291-1296), see
tests/test_oracle_golden.py::test_pybuilder_reproduces_reference_vectors.
"""


def internet_checksum(data, acc=0):
    """checksum.rs:5-29 (u32 wrap as in a release build)."""
    s = acc & 0xFFFFFFFF
    n = len(data)
    i = 0
    while n - i > 1:
        s = (s + ((data[i] << 8) | data[i + 1])) & 0xFFFFFFFF
        i += 2
    if n - i > 0:
        s = (s + (data[i] << 8)) & 0xFFFFFFFF
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def pseudo_header(src, dst, protocol, length):
    """checksum.rs:43-69."""
    s = 0
    for a in (src, dst):
        for k in range(0, len(a), 2):
            s += (a[k] << 8) | a[k + 1]
    return (s + protocol + length) & 0xFFFFFFFF


class Builder:
    """Mirrors PacketBuilder (builder.rs:55-90): a buffer and a header cursor."""

    def __init__(self, size):
        self.b = bytearray(size)
        self.hl = 0

    # -- datalink (ethernet.rs:19-129, builder.rs:110-221) ------------------
    def _eth_common(self, src, dst):
        self.b[0:6] = bytes(dst)
        self.b[6:12] = bytes(src)

    def ethernet(self, src, dst, ethertype):
        self._eth_common(src, dst)
        self.b[12] = (ethertype >> 8) & 0xFF
        self.b[13] = ethertype & 0xFF
        self.hl = 14
        return self

    def ethernet_vlan(self, src, dst, ethertype, tci):
        self._eth_common(src, dst)
        self.b[12:16] = bytes([0x81, 0x00, (tci >> 8) & 0xFF, tci & 0xFF])
        self.b[16] = (ethertype >> 8) & 0xFF
        self.b[17] = ethertype & 0xFF
        self.hl = 18
        return self

    def ethernet_qinq(self, src, dst, ethertype, tci1, tci2):
        self._eth_common(src, dst)
        self.b[12:20] = bytes([0x88, 0xA8, (tci1 >> 8) & 0xFF, tci1 & 0xFF,
                               0x81, 0x00, (tci2 >> 8) & 0xFF, tci2 & 0xFF])
        self.b[20] = (ethertype >> 8) & 0xFF
        self.b[21] = ethertype & 0xFF
        self.hl = 22
        return self

    def arp(self, htype, ptype, hlen, plen, oper, sha, spa, tha, tpa):
        """arp.rs:7-119, builder.rs:198-236."""
        o = self.hl
        self.b[o:o + 8] = bytes([htype >> 8, htype & 0xFF, ptype >> 8, ptype & 0xFF,
                                 hlen, plen, oper >> 8, oper & 0xFF])
        self.b[o + 8:o + 14] = bytes(sha)
        self.b[o + 14:o + 18] = bytes(spa)
        self.b[o + 18:o + 24] = bytes(tha)
        self.b[o + 24:o + 28] = bytes(tpa)
        self.hl += 28
        return self

    # -- network (ipv4.rs:8-127, ipv6.rs:8-133) ------------------------------
    def ipv4(self, version, ihl, dscp, ecn, total_length, ident, flags, frag_off,
             ttl, protocol, src, dst):
        o = self.hl
        b = self.b
        b[o] = (b[o] & 0x0F) | ((version << 4) & 0xFF)
        b[o] = (b[o] & 0xF0) | (ihl & 0x0F)
        b[o + 1] = (b[o + 1] & 0x03) | ((dscp << 2) & 0xFF)
        b[o + 1] = (b[o + 1] & 0xFC) | (ecn & 0x03)
        b[o + 2] = (total_length >> 8) & 0xFF
        b[o + 3] = total_length & 0xFF
        b[o + 4] = (ident >> 8) & 0xFF
        b[o + 5] = ident & 0xFF
        b[o + 6] = (b[o + 6] & 0x1F) | (((flags << 5) & 0xFF) & 0xE0)
        b[o + 6] = (b[o + 6] & 0xE0) | ((frag_off >> 8) & 0x1F)
        b[o + 7] = frag_off & 0xFF
        b[o + 8] = ttl
        b[o + 9] = protocol
        b[o + 12:o + 16] = bytes(src)
        b[o + 16:o + 20] = bytes(dst)
        # set_checksum (ipv4.rs:119-126)
        b[o + 10] = 0
        b[o + 11] = 0
        hl = (b[o] & 0x0F) * 4
        c = internet_checksum(b[o:o + hl], 0)
        b[o + 10] = c >> 8
        b[o + 11] = c & 0xFF
        self.hl += hl
        return self

    def ipv6(self, version, traffic_class, flow_label, payload_length, next_header,
             hop_limit, src, dst):
        o = self.hl
        b = self.b
        b[o] = (b[o] & 0x0F) | ((version << 4) & 0xFF)
        b[o] = (b[o] & 0xF0) | (traffic_class >> 4)
        b[o + 1] = (b[o + 1] & 0x0F) | ((traffic_class << 4) & 0xFF)
        b[o + 1] = (b[o + 1] & 0xF0) | ((flow_label >> 16) & 0xFF)
        b[o + 2] = (flow_label >> 8) & 0xFF
        b[o + 3] = flow_label & 0xFF
        b[o + 4] = (payload_length >> 8) & 0xFF
        b[o + 5] = payload_length & 0xFF
        b[o + 6] = next_header
        b[o + 7] = hop_limit
        b[o + 8:o + 24] = bytes(src)
        b[o + 24:o + 40] = bytes(dst)
        self.hl += 40
        return self

    # -- IPv6 extension headers (options.rs, routing.rs, fragment.rs,
    #    authentication.rs writers; builder.rs:607-806) ----------------------
    def _options(self, next_header, ext_len, options):
        o = self.hl
        self.b[o] = next_header
        self.b[o + 1] = ext_len
        assert len(options) >= 6 and len(options) == ext_len * 8
        self.b[o + 2:o + 2 + len(options)] = bytes(options)
        self.hl += (ext_len + 1) * 8
        return self

    def hop_by_hop(self, next_header, ext_len, options):
        return self._options(next_header, ext_len, options)

    def destination_options1(self, next_header, ext_len, options):
        return self._options(next_header, ext_len, options)

    def destination_options2(self, next_header, ext_len, options):
        return self._options(next_header, ext_len, options)

    def routing_header(self, next_header, ext_len, routing_type, segments_left, data):
        o = self.hl
        self.b[o:o + 4] = bytes([next_header, ext_len, routing_type, segments_left])
        assert len(data) >= 4 and len(data) == ext_len * 8
        self.b[o + 8:o + 8 + len(data)] = bytes(data)
        self.hl += (ext_len + 1) * 8
        return self

    def fragment_header(self, next_header, fragment_offset, m_flag, identification):
        o = self.hl
        b = self.b
        b[o] = next_header
        b[o + 1] = 0
        v = fragment_offset & 0x1FFF
        b[o + 2] = (v >> 5) & 0xFF
        b[o + 3] = (b[o + 3] & 0xE0) | (v & 0x1F)
        b[o + 3] = (b[o + 3] & 0x9F)
        b[o + 3] = (b[o + 3] | 0x80) if m_flag else (b[o + 3] & 0x7F)
        b[o + 4:o + 8] = identification.to_bytes(4, "big")
        self.hl += 8
        return self

    def authentication_header(self, next_header, payload_len, spi, seq, auth_data):
        o = self.hl
        b = self.b
        b[o] = next_header
        b[o + 1] = payload_len
        b[o + 2] = 0
        b[o + 3] = 0
        b[o + 4:o + 8] = spi.to_bytes(4, "big")
        b[o + 8:o + 12] = seq.to_bytes(4, "big")
        b[o + 12:o + 12 + len(auth_data)] = bytes(auth_data)
        self.hl += (payload_len + 2) * 4
        return self

    # -- transport (tcp.rs:7-130, udp.rs:7-92, icmpv4.rs:10-81, icmpv6.rs:7-78)
    def tcp(self, src_ip, src_port, dst_ip, dst_port, seq, ack, data_offset, reserved,
            flags, window, urgent, payload=None):
        o = self.hl
        b = self.b
        b[o:o + 4] = bytes([src_port >> 8, src_port & 0xFF, dst_port >> 8, dst_port & 0xFF])
        b[o + 4:o + 8] = (seq & 0xFFFFFFFF).to_bytes(4, "big")
        b[o + 8:o + 12] = (ack & 0xFFFFFFFF).to_bytes(4, "big")
        b[o + 12] = ((data_offset << 4) & 0xFF) | (b[o + 12] & 0x0F)
        b[o + 12] = (b[o + 12] & 0xF0) | (reserved & 0x0F)
        b[o + 13] = flags
        b[o + 14] = window >> 8
        b[o + 15] = window & 0xFF
        b[o + 18] = urgent >> 8
        b[o + 19] = urgent & 0xFF
        hl = (b[o + 12] >> 4) * 4
        if payload is not None:
            b[o + hl:o + hl + len(payload)] = bytes(payload)
        seg_len = len(b) - o
        b[o + 16] = 0
        b[o + 17] = 0
        c = internet_checksum(b[o:], pseudo_header(src_ip, dst_ip, 6, seg_len))
        b[o + 16] = c >> 8
        b[o + 17] = c & 0xFF
        self.hl += hl
        return self

    def udp(self, src_ip, src_port, dst_ip, dst_port, length, payload=None):
        o = self.hl
        b = self.b
        b[o:o + 6] = bytes([src_port >> 8, src_port & 0xFF, dst_port >> 8, dst_port & 0xFF,
                            length >> 8, length & 0xFF])
        if payload is not None:
            b[o + 8:o + 8 + len(payload)] = bytes(payload)
        seg_len = len(b) - o
        b[o + 6] = 0
        b[o + 7] = 0
        c = internet_checksum(b[o:], pseudo_header(src_ip, dst_ip, 17, seg_len))
        b[o + 6] = c >> 8
        b[o + 7] = c & 0xFF
        self.hl += 8
        return self

    def icmpv4(self, icmp_type, code, payload=None):
        o = self.hl
        b = self.b
        b[o] = icmp_type
        b[o + 1] = code
        if payload is not None:
            b[o + 8:o + 8 + len(payload)] = bytes(payload)
        b[o + 2] = 0
        b[o + 3] = 0
        c = internet_checksum(b[o:], 0)
        b[o + 2] = c >> 8
        b[o + 3] = c & 0xFF
        self.hl += 8
        return self

    def icmpv6(self, src, dst, icmp_type, code, payload=None):
        o = self.hl
        b = self.b
        b[o] = icmp_type
        b[o + 1] = code
        if payload is not None:
            b[o + 8:o + 8 + len(payload)] = bytes(payload)
        seg_len = len(b) - o
        b[o + 2] = 0
        b[o + 3] = 0
        c = internet_checksum(b[o:], pseudo_header(src, dst, 58, seg_len))
        b[o + 2] = c >> 8
        b[o + 3] = c & 0xFF
        self.hl += 8
        return self

    def build(self):
        return bytes(self.b)
