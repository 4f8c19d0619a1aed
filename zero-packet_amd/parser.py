"""PacketParser / *Reader facade over zp_record (the reference's public API).

Mirrors src/packet/parser.rs:22-69 and the reader views of src/datalink,
src/network and src/transport: field names, getters and `Result` errors
(raised as ZeroPacketError carrying the exact reference string). Every
reader is a view `frame[start:]` that runs to the end of the frame, exactly
like the reference's `&'a [u8]` sub-slices, so a PacketParser is rebuilt from
a record without re-parsing (PacketParser.from_record).

PacketParser.parse(frame) parses through the GPU (zp_parse_one); batches go
through zero-packet_amd.batch. There is no CPU parse path in this package.

The reference's direct reader use (README.md:110-115), `TcpReader::new(&pkt)?`,
is `TcpReader.new(pkt)`: the checked constructor of each reader, through
zp_reader_new (host code of libzp_hip.so; Ethernet also checks its VLAN
tagging, IPv6 runs the extension walk, ipv6.rs:159). It raises
ZeroPacketError with the reference's string. `XReader(bytes)` stays the
unchecked view that from_record builds. internet_checksum,
verify_internet_checksum and pseudo_header are checksum.rs:5,33,67 through
the same library.
"""
import atexit
import ctypes
import threading

import numpy as np

from . import _lib
from . import records as _rec
from .records import (EXT_DTYPE, EXT_SLOTS, F_ARP, F_ETHERNET, F_EXT, F_EXT_SLOT, F_ICMPV4,
                      F_ICMPV6, F_INNER_EXT, F_INNER_EXT_SLOT, F_IP_IN_IP, F_IP_IN_IP_V6,
                      F_IPV4, F_IPV6, F_TCP, F_UDP, READER_INFO_DTYPE, RECORD_DTYPE)


class ZeroPacketError(Exception):
    """Err(&'static str) of the reference; .code is the zp_err value."""

    def __init__(self, message, code=None):
        super().__init__(message)
        self.code = code


def _be16(b, i):
    return (b[i] << 8) | b[i + 1]


def _be32(b, i):
    return (b[i] << 24) | (b[i + 1] << 16) | (b[i + 2] << 8) | b[i + 3]


def _buf(data):
    data = bytes(data)
    return data, ctypes.create_string_buffer(data, max(len(data), 1))


def _py_internet_checksum(data, accumulator):
    """checksum.rs:5-29 in Python (used when libzp_hip.so cannot be loaded):
    big-endian words, an odd tail byte as the high byte, u32 wrap-around,
    fold, complement."""
    n = len(data) & ~1
    words = np.frombuffer(data[:n], dtype=">u2").astype(np.uint64)
    s = int(words.sum()) + accumulator + ((data[-1] << 8) if len(data) & 1 else 0)
    s &= 0xFFFFFFFF
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def internet_checksum(data, accumulator=0):
    """internet_checksum (checksum.rs:5-29) via zp_internet_checksum; the
    Python restatement when the library is not loadable (host helper, not
    the parse path)."""
    data, b = _buf(data)
    if not _lib_available():
        return _py_internet_checksum(data, accumulator & 0xFFFFFFFF)
    return int(_lib.hip().zp_internet_checksum(b, len(data), accumulator & 0xFFFFFFFF))


def verify_internet_checksum(data, accumulator=0):
    """verify_internet_checksum (checksum.rs:33-35)."""
    return internet_checksum(data, accumulator) == 0


def pseudo_header(src, dest, protocol, length):
    """pseudo_header (checksum.rs:38-69) of 4-byte or 16-byte addresses."""
    src, dest = bytes(src), bytes(dest)
    if len(src) != len(dest) or len(src) not in (4, 16):
        raise ValueError("pseudo_header: both addresses 4 bytes (IPv4) or 16 bytes (IPv6)")
    return int(_lib.hip().zp_pseudo_header(src, dest, len(src), protocol & 0xFF, length))


def _reader_new(kind, data):
    """zp_reader_new: the reference constructor's checks; raises its Err."""
    data, b = _buf(data)
    info = np.zeros(1, READER_INFO_DTYPE)
    rc = _lib.hip().zp_reader_new(kind, b, len(data), info.ctypes.data)
    if rc < 0:
        raise ValueError(f"zp_reader_new: bad arguments (kind {kind})")
    if rc:
        raise ZeroPacketError(_lib.hip().zp_err_str(rc).decode(), rc)
    return data, info[0]


class _Reader:
    KIND = None

    def __init__(self, data):
        self.bytes = bytes(data)

    def __eq__(self, other):
        return type(self) is type(other) and self.bytes == other.bytes

    @classmethod
    def new(cls, data):
        """XReader::new(&[u8]) -> Result: the checked constructor."""
        data, info = _reader_new(cls.KIND, data)
        return cls._from_info(data, info)

    @classmethod
    def _from_info(cls, data, info):
        return cls(data)


class EthernetReader(_Reader):
    """ethernet.rs:131-263. EthernetReader(data, header_len) is the view;
    EthernetReader.new(data) (or header_len=None) the checked constructor."""
    KIND = _rec.READER_ETHERNET

    def __init__(self, data, header_len=None):
        super().__init__(data)
        if header_len is None:
            if _lib_available():
                header_len = int(_reader_new(self.KIND, self.bytes)[1]["header_len"])
            else:                               # ethernet.rs:141-179 without the library
                if len(self.bytes) < 14:
                    raise ZeroPacketError("Slice is too short to contain an Ethernet frame.", 2)
                header_len = self.calculate_header_len(self.bytes)
        self._hl = header_len

    @classmethod
    def _from_info(cls, data, info):
        return cls(data, int(info["header_len"]))

    @staticmethod
    def calculate_header_len(b):
        t = _be16(b, 12)
        if t == 0x8100:
            if len(b) < 18:
                raise ZeroPacketError("Slice is too short to contain VLAN tagging.", 3)
            return 18
        if t == 0x88A8:
            if len(b) < 22:
                raise ZeroPacketError("Slice is too short to contain double VLAN tagging.", 4)
            if _be16(b, 16) != 0x8100:
                raise ZeroPacketError("Invalid double VLAN tag.", 5)
            return 22
        return 14

    @staticmethod
    def is_vlan_tagged(b):
        return _be16(b, 12) == 0x8100

    @staticmethod
    def is_vlan_double_tagged(b):
        return _be16(b, 12) == 0x88A8

    def dest_mac(self):
        return self.bytes[0:6]

    def src_mac(self):
        return self.bytes[6:12]

    def ethertype(self):
        return _be16(self.bytes, self._hl - 2)

    def vlan_tag(self):
        if not self.is_vlan_tagged(self.bytes):
            return None
        return (_be16(self.bytes, 12), _be16(self.bytes, 14))

    def double_vlan_tag(self):
        if not self.is_vlan_double_tagged(self.bytes):
            return None
        b = self.bytes
        return ((_be16(b, 12), _be16(b, 14)), (_be16(b, 16), _be16(b, 18)))

    def header_len(self):
        return self._hl

    def header(self):
        return self.bytes[:self._hl]

    def payload(self):
        return self.bytes[self._hl:]


class ArpReader(_Reader):
    """arp.rs:121-227."""
    KIND = _rec.READER_ARP

    def htype(self): return _be16(self.bytes, 0)
    def ptype(self): return _be16(self.bytes, 2)
    def hlen(self): return self.bytes[4]
    def plen(self): return self.bytes[5]
    def oper(self): return _be16(self.bytes, 6)
    def sha(self): return self.bytes[8:14]
    def spa(self): return self.bytes[14:18]
    def tha(self): return self.bytes[18:24]
    def tpa(self): return self.bytes[24:28]
    def header_len(self): return 28
    def header(self): return self.bytes[:28]
    def payload(self): return self.bytes[28:]


class IPv4Reader(_Reader):
    """ipv4.rs:129-265."""
    KIND = _rec.READER_IPV4

    def version(self): return self.bytes[0] >> 4
    def ihl(self): return self.bytes[0] & 0x0F
    def dscp(self): return self.bytes[1] >> 2
    def ecn(self): return self.bytes[1] & 0x03
    def total_length(self): return _be16(self.bytes, 2)
    def id(self): return _be16(self.bytes, 4)
    def flags(self): return self.bytes[6] >> 5
    def fragment_offset(self): return ((self.bytes[6] & 0x1F) << 8) | self.bytes[7]
    def ttl(self): return self.bytes[8]
    def protocol(self): return self.bytes[9]
    def src_ip(self): return self.bytes[12:16]
    def dest_ip(self): return self.bytes[16:20]
    def checksum(self): return _be16(self.bytes, 10)
    def header_len(self): return self.ihl() * 4

    def header(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError("Indicated IPv4 header length exceeds the allocated buffer.", 14)
        return self.bytes[:self.header_len()]

    def payload(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError("Indicated IPv4 header length exceeds the allocated buffer.", 14)
        return self.bytes[self.header_len():]

    def valid_checksum(self):
        """ipv4.rs:262-264: raises when header() does."""
        return internet_checksum(self.header(), 0) == 0


class OptionsHeaderReader(_Reader):
    """extensions/options.rs:76-154 (Hop-by-Hop / Destination Options)."""
    KIND = _rec.READER_OPTIONS

    def next_header(self): return self.bytes[0]
    def header_ext_len(self): return self.bytes[1]
    def header_len(self): return (self.bytes[1] + 1) * 8

    def options(self):
        if len(self.bytes) < self.header_len():
            raise ZeroPacketError("Indicated header length exceeds the allocated buffer.", 37)
        return self.bytes[2:self.header_len()]

    def header(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError(
                "Indicated IPv6 options header length exceeds the allocated buffer.", 19)
        return self.bytes[:self.header_len()]

    def payload(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError(
                "Indicated IPv6 options header length exceeds the allocated buffer.", 19)
        return self.bytes[self.header_len():]


class RoutingHeaderReader(_Reader):
    """extensions/routing.rs:99-195."""
    KIND = _rec.READER_ROUTING

    def next_header(self): return self.bytes[0]
    def header_ext_len(self): return self.bytes[1]
    def routing_type(self): return self.bytes[2]
    def segments_left(self): return self.bytes[3]
    def data(self):
        """routing.rs:156-161 slices unchecked: the reference panics when the
        header runs past the slice; IndexError here."""
        if self.header_len() > len(self.bytes):
            raise IndexError("RoutingHeaderReader.data: header past the slice")
        return self.bytes[4:self.header_len()]
    def header_len(self): return (self.bytes[1] + 1) * 8

    def header(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError(
                "Indicated IPv6 routing header length exceeds the allocated buffer.", 21)
        return self.bytes[:self.header_len()]

    def payload(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError(
                "Indicated IPv6 routing header length exceeds the allocated buffer.", 21)
        return self.bytes[self.header_len():]


class FragmentHeaderReader(_Reader):
    """extensions/fragment.rs:90-173."""
    KIND = _rec.READER_FRAGMENT

    def next_header(self): return self.bytes[0]
    def reserved(self): return self.bytes[1]
    def fragment_offset(self): return (self.bytes[2] << 5) | (self.bytes[3] & 0x1F)
    def res(self): return (self.bytes[3] >> 5) & 0b11
    def m_flag(self): return (self.bytes[3] & 0x80) != 0
    def identification(self): return _be32(self.bytes, 4)
    def header_len(self): return 8
    def header(self): return self.bytes[:8]
    def payload(self): return self.bytes[8:]


class AuthenticationHeaderReader(_Reader):
    """extensions/authentication.rs:97-200."""
    KIND = _rec.READER_AUTH

    def next_header(self): return self.bytes[0]
    def payload_len(self): return self.bytes[1]
    def reserved(self): return _be16(self.bytes, 2)
    def spi(self): return _be32(self.bytes, 4)
    def sequence_number(self): return _be32(self.bytes, 8)
    def header_len(self): return (self.bytes[1] + 2) * 4

    def authentication_data(self):
        """authentication.rs:161-169; a header_len below 12 (payload_len 0 or
        1) makes the reference's bytes[12..header_len] panic: IndexError."""
        if len(self.bytes) < self.header_len():
            raise ZeroPacketError(
                "Indicated Authentication header length exceeds the allocated buffer.", 24)
        if self.header_len() < 12:
            raise IndexError("AuthenticationHeaderReader.authentication_data: header_len < 12")
        return self.bytes[12:self.header_len()]

    def header(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError(
                "Indicated Authentication header length exceeds the allocated buffer.", 24)
        return self.bytes[:self.header_len()]

    def payload(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError(
                "Indicated Authentication header length exceeds the allocated buffer.", 24)
        return self.bytes[self.header_len():]


_EXT_CLS = [OptionsHeaderReader, RoutingHeaderReader, FragmentHeaderReader,
            AuthenticationHeaderReader, OptionsHeaderReader, OptionsHeaderReader]


class ExtensionHeaders:
    """extensions/headers.rs:19-28."""

    def __init__(self):
        self.hop_by_hop = self.routing = self.fragment = None
        self.auth_header = self.destination_1st = self.destination_2nd = None
        self.total_headers_len = 0
        self.final_next_header = 0


class IPv6Reader(_Reader):
    """ipv6.rs:135-286. Built from a record: extension headers come from the
    record's offsets instead of a re-walk. IPv6Reader.new(data) runs the walk
    (ipv6.rs:147-167)."""
    KIND = _rec.READER_IPV6

    def __init__(self, data, extension_headers=None, extension_headers_len=0):
        super().__init__(data)
        self.extension_headers = extension_headers
        self.extension_headers_len = extension_headers_len

    @classmethod
    def _from_info(cls, data, info):
        flags = int(info["flags"])
        if not flags & F_EXT:
            return cls(data)
        x = info["ext"]
        eh = _ext_from(data, 40, flags, 12, x["off"], x["len"], info["final_nh"])
        return cls(data, eh, int(x["len"]))

    def version(self): return self.bytes[0] >> 4
    def traffic_class(self): return ((self.bytes[0] & 0x0F) << 4) | (self.bytes[1] >> 4)

    def flow_label(self):
        return ((self.bytes[1] & 0x0F) << 16) | (self.bytes[2] << 8) | self.bytes[3]

    def payload_length(self): return _be16(self.bytes, 4)
    def next_header(self): return self.bytes[6]

    def final_next_header(self):
        if self.extension_headers is not None:
            return self.extension_headers.final_next_header
        return self.next_header()

    def hop_limit(self): return self.bytes[7]
    def src_addr(self): return self.bytes[8:24]
    def dest_addr(self): return self.bytes[24:40]
    def header_len(self): return 40
    def header(self): return self.bytes[:40]
    def payload(self): return self.bytes[40:]
    def upper_layer_payload(self): return self.bytes[40 + self.extension_headers_len:]


class TcpReader(_Reader):
    """tcp.rs:132-244."""
    KIND = _rec.READER_TCP

    def src_port(self): return _be16(self.bytes, 0)
    def dest_port(self): return _be16(self.bytes, 2)
    def sequence_number(self): return _be32(self.bytes, 4)
    def ack_number(self): return _be32(self.bytes, 8)
    def data_offset(self): return self.bytes[12] >> 4
    def reserved(self): return self.bytes[12] & 0x0F
    def flags(self): return self.bytes[13]
    def window_size(self): return _be16(self.bytes, 14)
    def checksum(self): return _be16(self.bytes, 16)
    def urgent_pointer(self): return _be16(self.bytes, 18)
    def header_len(self): return self.data_offset() * 4

    def header(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError("Indicated TCP header length exceeds the allocated buffer.", 36)
        return self.bytes[:self.header_len()]

    def payload(self):
        if self.header_len() > len(self.bytes):
            raise ZeroPacketError("Indicated TCP header length exceeds the allocated buffer.", 36)
        return self.bytes[self.header_len():]


class UdpReader(_Reader):
    """udp.rs:94-154."""
    KIND = _rec.READER_UDP

    def src_port(self): return _be16(self.bytes, 0)
    def dest_port(self): return _be16(self.bytes, 2)
    def checksum(self): return _be16(self.bytes, 6)
    def length(self): return _be16(self.bytes, 4)
    def header_len(self): return 8
    def header(self): return self.bytes[:8]
    def payload(self): return self.bytes[8:]


class _IcmpReader(_Reader):
    def icmp_type(self): return self.bytes[0]
    def icmp_code(self): return self.bytes[1]
    def checksum(self): return _be16(self.bytes, 2)
    def header_len(self): return 8
    def header(self): return self.bytes[:8]
    def payload(self): return self.bytes[8:]


class Icmpv4Reader(_IcmpReader):
    """icmpv4.rs:83-135."""
    KIND = _rec.READER_ICMPV4


class Icmpv6Reader(_IcmpReader):
    """icmpv6.rs:80-132."""
    KIND = _rec.READER_ICMPV6


class IpInIp:
    """misc.rs:6-9: IpInIp::Ipv4(IPv4Reader) | IpInIp::Ipv6(IPv6Reader)."""

    def __init__(self, kind, reader):
        self.kind = kind          # "ipv4" or "ipv6"
        self.reader = reader

    def __repr__(self):
        return f"IpInIp::{'Ipv4' if self.kind == 'ipv4' else 'Ipv6'}"


def _ext_from(frame, payload_off, flags, shift, offs, total, final_nh):
    eh = ExtensionHeaders()
    for k, name in enumerate(EXT_SLOTS):
        if flags & (1 << (shift + k)):
            setattr(eh, name, _EXT_CLS[k](frame[payload_off + int(offs[k]):]))
    eh.total_headers_len = int(total)
    eh.final_next_header = int(final_nh)
    return eh


class PacketParser:
    """parser.rs:22-32. Fields are None or reader views."""

    FIELDS = ("ethernet", "arp", "ipv4", "ipv6", "ip_in_ip", "tcp", "udp", "icmpv4", "icmpv6")
    # the absent fields: class-level None, so building a parser sets only the
    # readers present (a per-instance loop over FIELDS cost ~1 us per frame
    # of PacketParser.parse)
    ethernet = arp = ipv4 = ipv6 = ip_in_ip = tcp = udp = icmpv4 = icmpv6 = None

    @classmethod
    def from_record(cls, frame, rec, ext=None):
        """Rebuilds the parser of `frame` from its zp_record (no re-parse).
        ext: the frame's two zp_ext_offsets entries (outer ipv6 chain,
        ip_in_ip chain; EXT_DTYPE [2]), needed when the record flags a chain.
        Raises ZeroPacketError when the record holds an error."""
        frame = bytes(frame)
        word = int(rec["flags"])
        err = word >> 26
        if err:
            raise ZeroPacketError(_lib.hip().zp_err_str(err).decode() if _lib_available()
                                  else f"zp_err {err}", err)
        flags = word & _rec.F_MASK
        if _rec.chain_inline(rec):                 # ABI v6: the outer chain in the record
            ext = _rec.expand_ext(np.array([(rec["flags"], rec["offs"])], RECORD_DTYPE),
                                  np.zeros(2, EXT_DTYPE) if ext is None else ext).reshape(2)
        if flags & (F_EXT | F_INNER_EXT) and ext is None:
            raise ValueError("the record flags an IPv6 extension chain: pass its ext entries")
        # both record forms (the far-L4 one reads eth_len / inner_off from the frame)
        d = _rec.decode(frame, rec, ext)
        p = cls()
        hl, io, l4 = d["eth_len"], d["inner_off"], d["l4_off"]
        if flags & F_ETHERNET:
            p.ethernet = EthernetReader(frame, hl)
        if flags & F_ARP:
            p.arp = ArpReader(frame[hl:])
        if flags & F_IPV4:
            p.ipv4 = IPv4Reader(frame[hl:])
        if flags & F_IPV6:
            eh = None
            if flags & F_EXT:
                x = ext[0]
                eh = _ext_from(frame, hl + 40, flags, 12, x["off"], x["len"], x["final_nh"])
            p.ipv6 = IPv6Reader(frame[hl:], eh, int(ext[0]["len"]) if eh else 0)
        if flags & F_IP_IN_IP:
            if flags & F_IP_IN_IP_V6:
                eh = None
                if flags & F_INNER_EXT:
                    x = ext[1]
                    eh = _ext_from(frame, io + 40, flags, 18, x["off"], x["len"], x["final_nh"])
                p.ip_in_ip = IpInIp("ipv6", IPv6Reader(frame[io:], eh,
                                                       int(ext[1]["len"]) if eh else 0))
            else:
                p.ip_in_ip = IpInIp("ipv4", IPv4Reader(frame[io:]))
        if flags & F_TCP:
            p.tcp = TcpReader(frame[l4:])
        if flags & F_UDP:
            p.udp = UdpReader(frame[l4:])
        if flags & F_ICMPV4:
            p.icmpv4 = Icmpv4Reader(frame[l4:])
        if flags & F_ICMPV6:
            p.icmpv6 = Icmpv6Reader(frame[l4:])
        return p

    def debug(self, pretty=False):
        """format!("{:?}") / format!("{:#?}") of the reference (debugfmt.py)."""
        from .debugfmt import debug
        return debug(self, pretty)

    @classmethod
    def parse(cls, frame):
        """PacketParser::parse (parser.rs:53) through the GPU path, on the
        calling thread's current HIP device. Reentrant like the reference's
        pure parse: each call takes a context of its own from the device's
        pool (a zp_ctx serves one call at a time), with no global lock. A
        frame of <= 64 KiB is answered by the context's resident server in
        ~4.5 us with the GIL held (cheaper than a GIL hand-off, _lib.pyhip);
        longer frames take the batch path with the GIL released."""
        frame = bytes(frame)
        n = len(frame)
        pyhip = _lib.pyhip()
        dev = pyhip.zp_device_current()
        if dev < 0:
            raise RuntimeError("zp_device_current failed: " + _lib.hip().zp_last_error().decode())
        pool = _POOLS.get(dev) or _pool(dev)
        if n <= ONE_MAX:
            # through the resident server: the GIL stays held (_lib.pyhip);
            # the record lands in the context's own buffers, read before the
            # context goes back to the pool
            ctx = pool.take()
            try:
                b = pool.bufs.get(ctx) or pool.buffers(ctx)
                rc = pyhip.zp_parse_one(ctx, frame, n, b[2], b[3])
                if rc >= 0:
                    return cls._from_words(frame, b[0][0], b[0][1], b[1])
            finally:
                pool.give(ctx)
            _lib.check(rc, "zp_parse_one")
        rec = (ctypes.c_uint32 * 2)()
        ext = (ctypes.c_uint8 * (2 * _rec.EXT_BYTES))()
        with pool.big_context() as ctx:
            rc = _lib.hip().zp_parse_one(ctx, frame, n, ctypes.addressof(rec),
                                         ctypes.addressof(ext))
        if rc < 0:
            _lib.check(rc, "zp_parse_one")
        return cls._from_words(frame, rec[0], rec[1], ext)

    @classmethod
    def _from_words(cls, frame, w, o, ext):
        """from_record for the record words (w, o) of zp_parse_one; the
        ordinary form without extension chains directly (the common frame),
        every other record through from_record."""
        flags = w & _rec.F_MASK
        if w >> 26 or flags & (F_EXT | F_INNER_EXT) or (w >> 24) & 3 == _rec.ETH_CODE_FAR:
            return cls.from_record(frame, np.array([(w, o)], RECORD_DTYPE)[0],
                                   np.frombuffer(bytes(ext), EXT_DTYPE))
        hl = 14 + 4 * ((w >> 24) & 3)                      # records.decode, ordinary form
        l4 = o & _rec.L4_NEAR_MAX
        p = cls()
        if flags & F_ETHERNET:
            p.ethernet = EthernetReader(frame, hl)
        if flags & F_ARP:
            p.arp = ArpReader(frame[hl:])
        if flags & F_IPV4:
            p.ipv4 = IPv4Reader(frame[hl:])
        if flags & F_IPV6:
            p.ipv6 = IPv6Reader(frame[hl:], None, 0)
        if flags & F_IP_IN_IP:
            io = o >> 18
            if flags & F_IP_IN_IP_V6:
                p.ip_in_ip = IpInIp("ipv6", IPv6Reader(frame[io:], None, 0))
            else:
                p.ip_in_ip = IpInIp("ipv4", IPv4Reader(frame[io:]))
        if flags & F_TCP:
            p.tcp = TcpReader(frame[l4:])
        if flags & F_UDP:
            p.udp = UdpReader(frame[l4:])
        if flags & F_ICMPV4:
            p.icmpv4 = Icmpv4Reader(frame[l4:])
        if flags & F_ICMPV6:
            p.icmpv6 = Icmpv6Reader(frame[l4:])
        return p


def _lib_available():
    try:
        _lib.hip()
        return True
    except Exception:
        return False


ONE_MAX = 64 << 10          # zp_parse_one's mapped-block frame limit (zp_ctx.hip ONE_MAX)
POOL_CHUNK = 1 << 20        # chunk size of a pooled context (frames <= ONE_MAX only)
POOL_MAX = 32               # pooled contexts per device; more callers wait for one


class _DevicePool:
    """zp_ctx pool of one device. Frames up to ONE_MAX take a small pooled
    context each (its own mapped block and slot in the device's resident
    server, so calls on different threads never wait for each other);
    longer frames take the device's one large context (256 MiB chunks)
    under a lock."""

    def __init__(self, device):
        self.device = device
        self.cv = threading.Condition()
        self.free = []
        self.all = []
        self.waiting = 0
        self.big = None
        self.big_lock = threading.Lock()
        self.bufs = {}                          # pooled context -> its record / ext buffers

    def buffers(self, ctx):
        """The record and ext buffers of pooled context `ctx` (and their
        addresses), made on its first call; only the caller holding ctx
        touches them."""
        rec = (ctypes.c_uint32 * 2)()
        ext = (ctypes.c_uint8 * (2 * _rec.EXT_BYTES))()
        b = self.bufs[ctx] = (rec, ext, ctypes.addressof(rec), ctypes.addressof(ext))
        return b

    def _create(self, chunk):
        lib = _lib.hip()
        ctx = lib.zp_ctx_create(self.device, chunk)
        if not ctx:
            raise RuntimeError("zp_ctx_create failed: " + lib.zp_last_error().decode())
        return ctx

    def take(self):
        """A free pooled context (created when none is free and the pool is
        below POOL_MAX; else the caller waits for one)."""
        try:
            return self.free.pop()              # LIFO: the context whose server is warm
        except IndexError:
            pass
        with self.cv:
            while not self.free and len(self.all) >= POOL_MAX:
                self.waiting += 1
                self.cv.wait()
                self.waiting -= 1
            if self.free:
                return self.free.pop()
            self.all.append(None)               # reserve a slot, create outside the lock
        try:
            ctx = self._create(POOL_CHUNK)
        except Exception:
            with self.cv:
                self.all.remove(None)
                self.cv.notify()
            raise
        with self.cv:
            self.all[self.all.index(None)] = ctx
        return ctx

    def give(self, ctx):
        self.free.append(ctx)                   # list append / pop are atomic under the GIL
        if self.waiting:
            with self.cv:
                self.cv.notify()

    class _BigLease:
        def __init__(self, pool):
            self.pool = pool

        def __enter__(self):
            p = self.pool
            p.big_lock.acquire()
            try:
                if p.big is None:
                    p.big = p._create(0)
            except Exception:
                p.big_lock.release()
                raise
            return p.big

        def __exit__(self, *exc):
            self.pool.big_lock.release()
            return False

    def big_context(self):
        """A lease on the device's large context (frames past ONE_MAX)."""
        return _DevicePool._BigLease(self)

    def quiesce(self):
        """Stops the servers of the contexts no call holds (a held one's
        server leaves within its 1 ms life anyway): they are taken out of
        the free list while their servers stop, then returned."""
        lib = _lib.hip()
        taken = []
        while True:
            try:
                taken.append(self.free.pop())
            except IndexError:
                break
        try:
            for ctx in taken:
                lib.zp_parse_one_config(ctx, 5000)
        finally:
            for ctx in taken:
                self.give(ctx)
        with self.big_lock:
            if self.big is not None:
                lib.zp_parse_one_config(self.big, 5000)


_POOLS = {}
_POOLS_LOCK = threading.Lock()


def _pool(device):
    """The context pool of `device` (created on first use)."""
    with _POOLS_LOCK:
        p = _POOLS.get(device)
        if p is None:
            if not _POOLS:
                atexit.register(quiesce)
            p = _POOLS[device] = _DevicePool(device)
        return p


def quiesce():
    """Stops the devices' resident zp_parse_one servers now, through the
    idle contexts of the pools (a server also leaves by itself after 1 ms
    resident whatever the traffic; the next PacketParser.parse relaunches
    it). Call before a device-wide synchronisation to avoid waiting for
    that bound."""
    with _POOLS_LOCK:
        pools = list(_POOLS.values())
    for p in pools:
        p.quiesce()
