// zero_packet.hpp — C++17 facade over the C ABI (include/zero_packet.h) that
// mirrors the reference's public parse API:
//
//   PacketParser::parse(&[u8]) -> Result<PacketParser, &'static str>
//                                       (/root/reference/src/packet/parser.rs:53)
//   struct PacketParser { ethernet, arp, ipv4, ipv6, ip_in_ip, tcp, udp,
//                         icmpv4, icmpv6 }   (parser.rs:22-32)
//   the *Reader views and their getters      (src/datalink, src/network,
//                                             src/transport)
//
// Every reader is a view `frame[start..]` that runs to the end of the frame,
// like the reference's `&'a [u8]` sub-slices (zero copy; the frame must
// outlive the views). A PacketParser is rebuilt from a zp_record without
// re-parsing (PacketParser::from_record). Errors are zp::Error carrying the
// zp_err code and the exact reference string. Header-only; parse() and the
// batch calls need libzp_hip.so (the GPU path), from_record() does not.
//
// The readers' checked constructors XReader::new(&[u8]) -> Result (the
// reference's direct use, README.md:110-115) are XReader::create(Bytes),
// which throws zp::Error on the reference's Err, and XReader::try_create
// (Bytes, int* err), which returns std::nullopt and the code instead (`new`
// is a C++ keyword). They go through zp_reader_new (libzp_hip.so; host
// code, no device), as do zp::internet_checksum / verify_internet_checksum /
// pseudo_header (checksum.rs:5,33,67). The explicit XReader(Bytes) view
// constructors stay unchecked, as from_record needs them.
#ifndef ZERO_PACKET_HPP
#define ZERO_PACKET_HPP

#include <array>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "zero_packet.h"
#include "zero_packet_errstr.h"

namespace zp {

// The `&'static str` of the reference's Err, with its zp_err code.
class Error : public std::runtime_error {
public:
    Error(int code, const char* msg) : std::runtime_error(msg ? msg : "zero-packet error"),
                                       code_(code) {}
    int code() const { return code_; }
private:
    int code_;
};

// A borrowed byte slice (&'a [u8]).
struct Bytes {
    const uint8_t* ptr = nullptr;
    size_t len = 0;
    size_t size() const { return len; }
    const uint8_t& operator[](size_t i) const { return ptr[i]; }
    Bytes sub(size_t from) const { return from <= len ? Bytes{ptr + from, len - from} : Bytes{ptr + len, 0}; }
    Bytes sub(size_t from, size_t to) const { return Bytes{ptr + from, to - from}; }
};

namespace detail {
inline uint16_t be16(Bytes b, size_t i) { return (uint16_t)((b[i] << 8) | b[i + 1]); }
inline uint32_t be32(Bytes b, size_t i) {
    return ((uint32_t)b[i] << 24) | ((uint32_t)b[i + 1] << 16) | ((uint32_t)b[i + 2] << 8) | b[i + 3];
}
template <size_t N> std::array<uint8_t, N> arr(Bytes b, size_t i) {
    std::array<uint8_t, N> a{};
    for (size_t k = 0; k < N; ++k) a[k] = b[i + k];
    return a;
}
[[noreturn]] inline void fail(int code) { throw Error(code, zp_err_string(code)); }

// XReader::new through the C ABI: std::nullopt and *err on the reference's Err.
template <class R>
std::optional<R> try_new(Bytes b, int* err) {
    zp_reader_info info;
    const int rc = zp_reader_new(R::kKind, b.ptr, b.len, &info);
    if (rc < 0) throw std::invalid_argument("zp_reader_new: null slice or unknown reader");
    if (err) *err = rc;
    if (rc != ZP_OK) return std::nullopt;
    return R::from_info(b, info);
}

// The checked constructors every reader shares (CRTP): `create` throws
// zp::Error with the reference's string, `try_create` returns std::nullopt.
// A reader with more state than its slice (Ethernet, IPv6) has its own
// from_info.
template <class R, int K>
struct Checked {
    static constexpr int kKind = K;
    static R from_info(Bytes b, const zp_reader_info&) { return R(b); }
    static R create(Bytes b) {
        int err = 0;
        std::optional<R> r = try_new<R>(b, &err);
        if (!r) fail(err);
        return *r;
    }
    static std::optional<R> try_create(Bytes b, int* err = nullptr) { return try_new<R>(b, err); }
};
}  // namespace detail

// checksum.rs:5-29 / :33-35 / :38-69 (the C ABI's host implementations).
inline uint16_t internet_checksum(Bytes data, uint32_t accumulator) {
    return zp_internet_checksum(data.ptr, data.len, accumulator);
}
inline bool verify_internet_checksum(Bytes data, uint32_t accumulator) {
    return zp_verify_internet_checksum(data.ptr, data.len, accumulator) != 0;
}
inline uint32_t pseudo_header(const std::array<uint8_t, 4>& src, const std::array<uint8_t, 4>& dest,
                              uint8_t protocol, size_t length) {
    return zp_pseudo_header(src.data(), dest.data(), 4, protocol, length);
}
inline uint32_t pseudo_header(const std::array<uint8_t, 16>& src, const std::array<uint8_t, 16>& dest,
                              uint8_t protocol, size_t length) {
    return zp_pseudo_header(src.data(), dest.data(), 16, protocol, length);
}

// ethernet.rs:131-263
class EthernetReader : public detail::Checked<EthernetReader, ZP_READER_ETHERNET> {
public:
    Bytes bytes;
    EthernetReader(Bytes b, size_t header_len) : bytes(b), hl_(header_len) {}
    // ethernet.rs:141-179: also the VLAN tagging checks
    static EthernetReader from_info(Bytes b, const zp_reader_info& i) {
        return EthernetReader(b, i.header_len);
    }
    std::array<uint8_t, 6> dest_mac() const { return detail::arr<6>(bytes, 0); }
    std::array<uint8_t, 6> src_mac() const { return detail::arr<6>(bytes, 6); }
    uint16_t ethertype() const { return detail::be16(bytes, hl_ - 2); }
    bool is_vlan_tagged() const { return detail::be16(bytes, 12) == 0x8100; }
    bool is_vlan_double_tagged() const { return detail::be16(bytes, 12) == 0x88A8; }
    // (tpid, tci) of a single 802.1Q tag (ethernet.rs:218-227)
    std::optional<std::pair<uint16_t, uint16_t>> vlan_tag() const {
        if (!is_vlan_tagged()) return std::nullopt;
        return std::make_pair(detail::be16(bytes, 12), detail::be16(bytes, 14));
    }
    // ((tpid, tci), (tpid, tci)) of a Q-in-Q pair (ethernet.rs:233-244)
    std::optional<std::pair<std::pair<uint16_t, uint16_t>, std::pair<uint16_t, uint16_t>>>
    double_vlan_tag() const {
        if (!is_vlan_double_tagged()) return std::nullopt;
        return std::make_pair(std::make_pair(detail::be16(bytes, 12), detail::be16(bytes, 14)),
                              std::make_pair(detail::be16(bytes, 16), detail::be16(bytes, 18)));
    }
    size_t header_len() const { return hl_; }
    Bytes header() const { return bytes.sub(0, hl_); }
    Bytes payload() const { return bytes.sub(hl_); }
private:
    size_t hl_;
};

// arp.rs:121-227
class ArpReader : public detail::Checked<ArpReader, ZP_READER_ARP> {
public:
    Bytes bytes;
    explicit ArpReader(Bytes b) : bytes(b) {}
    uint16_t htype() const { return detail::be16(bytes, 0); }
    uint16_t ptype() const { return detail::be16(bytes, 2); }
    uint8_t hlen() const { return bytes[4]; }
    uint8_t plen() const { return bytes[5]; }
    uint16_t oper() const { return detail::be16(bytes, 6); }
    std::array<uint8_t, 6> sha() const { return detail::arr<6>(bytes, 8); }
    std::array<uint8_t, 4> spa() const { return detail::arr<4>(bytes, 14); }
    std::array<uint8_t, 6> tha() const { return detail::arr<6>(bytes, 18); }
    std::array<uint8_t, 4> tpa() const { return detail::arr<4>(bytes, 24); }
    size_t header_len() const { return 28; }
    Bytes header() const { return bytes.sub(0, 28); }
    Bytes payload() const { return bytes.sub(28); }
};

// ipv4.rs:129-265
class IPv4Reader : public detail::Checked<IPv4Reader, ZP_READER_IPV4> {
public:
    Bytes bytes;
    explicit IPv4Reader(Bytes b) : bytes(b) {}
    uint8_t version() const { return bytes[0] >> 4; }
    uint8_t ihl() const { return bytes[0] & 0x0F; }
    uint8_t dscp() const { return bytes[1] >> 2; }
    uint8_t ecn() const { return bytes[1] & 0x03; }
    uint16_t total_length() const { return detail::be16(bytes, 2); }
    uint16_t id() const { return detail::be16(bytes, 4); }
    uint8_t flags() const { return bytes[6] >> 5; }
    uint16_t fragment_offset() const { return (uint16_t)(((bytes[6] & 0x1F) << 8) | bytes[7]); }
    uint8_t ttl() const { return bytes[8]; }
    uint8_t protocol() const { return bytes[9]; }
    uint16_t checksum() const { return detail::be16(bytes, 10); }
    std::array<uint8_t, 4> src_ip() const { return detail::arr<4>(bytes, 12); }
    std::array<uint8_t, 4> dest_ip() const { return detail::arr<4>(bytes, 16); }
    size_t header_len() const { return (size_t)ihl() * 4; }
    Bytes header() const { check(); return bytes.sub(0, header_len()); }
    Bytes payload() const { check(); return bytes.sub(header_len()); }
    // ipv4.rs:262-264: Err when header() is, else the header checksum
    bool valid_checksum() const { return internet_checksum(header(), 0) == 0; }
private:
    void check() const {   // ipv4.rs:238-241,252-255
        if (header_len() > bytes.size())
            detail::fail(ZP_ERR_IPV4_HDR_EXCEEDS);
    }
};

// extensions/options.rs:76-154 (Hop-by-Hop, Destination Options)
class OptionsHeaderReader : public detail::Checked<OptionsHeaderReader, ZP_READER_OPTIONS> {
public:
    Bytes bytes;
    explicit OptionsHeaderReader(Bytes b) : bytes(b) {}
    uint8_t next_header() const { return bytes[0]; }
    uint8_t header_ext_len() const { return bytes[1]; }
    size_t header_len() const { return ((size_t)bytes[1] + 1) * 8; }
    Bytes options() const {   // options.rs:111-119
        if (bytes.size() < header_len()) detail::fail(ZP_ERR_OPTIONS_DATA_EXCEEDS);
        return bytes.sub(2, header_len());
    }
    Bytes header() const { check(); return bytes.sub(0, header_len()); }
    Bytes payload() const { check(); return bytes.sub(header_len()); }
private:
    void check() const {
        if (header_len() > bytes.size())
            detail::fail(ZP_ERR_EXT_OPTIONS_EXCEEDS);
    }
};

// extensions/routing.rs:99-195
class RoutingHeaderReader : public detail::Checked<RoutingHeaderReader, ZP_READER_ROUTING> {
public:
    Bytes bytes;
    explicit RoutingHeaderReader(Bytes b) : bytes(b) {}
    uint8_t next_header() const { return bytes[0]; }
    uint8_t header_ext_len() const { return bytes[1]; }
    uint8_t routing_type() const { return bytes[2]; }
    uint8_t segments_left() const { return bytes[3]; }
    // routing.rs:156-161 slices bytes[4..header_len] unchecked: the reference
    // panics past the slice; this throws std::out_of_range there
    Bytes data() const {
        if (header_len() > bytes.size()) throw std::out_of_range("RoutingHeaderReader::data");
        return bytes.sub(4, header_len());
    }
    size_t header_len() const { return ((size_t)bytes[1] + 1) * 8; }
    Bytes header() const { check(); return bytes.sub(0, header_len()); }
    Bytes payload() const { check(); return bytes.sub(header_len()); }
private:
    void check() const {
        if (header_len() > bytes.size())
            detail::fail(ZP_ERR_EXT_ROUTING_EXCEEDS);
    }
};

// extensions/fragment.rs:90-173
class FragmentHeaderReader : public detail::Checked<FragmentHeaderReader, ZP_READER_FRAGMENT> {
public:
    Bytes bytes;
    explicit FragmentHeaderReader(Bytes b) : bytes(b) {}
    uint8_t next_header() const { return bytes[0]; }
    uint8_t reserved() const { return bytes[1]; }
    uint16_t fragment_offset() const { return (uint16_t)((bytes[2] << 5) | (bytes[3] & 0x1F)); }
    uint8_t res() const { return (bytes[3] >> 5) & 0x3; }
    bool m_flag() const { return (bytes[3] & 0x80) != 0; }
    uint32_t identification() const { return detail::be32(bytes, 4); }
    size_t header_len() const { return 8; }
    Bytes header() const { return bytes.sub(0, 8); }
    Bytes payload() const { return bytes.sub(8); }
};

// extensions/authentication.rs:97-200
class AuthenticationHeaderReader
    : public detail::Checked<AuthenticationHeaderReader, ZP_READER_AUTH> {
public:
    Bytes bytes;
    explicit AuthenticationHeaderReader(Bytes b) : bytes(b) {}
    uint8_t next_header() const { return bytes[0]; }
    uint8_t payload_len() const { return bytes[1]; }
    uint16_t reserved() const { return detail::be16(bytes, 2); }
    uint32_t spi() const { return detail::be32(bytes, 4); }
    uint32_t sequence_number() const { return detail::be32(bytes, 8); }
    size_t header_len() const { return ((size_t)bytes[1] + 2) * 4; }
    // authentication.rs:161-169; bytes[12..header_len] with header_len < 12
    // (payload_len 0 or 1) panics in the reference: std::out_of_range here
    Bytes authentication_data() const {
        check();
        if (header_len() < 12) throw std::out_of_range("AuthenticationHeaderReader::authentication_data");
        return bytes.sub(12, header_len());
    }
    Bytes header() const { check(); return bytes.sub(0, header_len()); }
    Bytes payload() const { check(); return bytes.sub(header_len()); }
private:
    void check() const {
        if (header_len() > bytes.size())
            detail::fail(ZP_ERR_EXT_AUTH_EXCEEDS);
    }
};

// extensions/headers.rs:19-28
struct ExtensionHeaders {
    std::optional<OptionsHeaderReader> hop_by_hop;
    std::optional<RoutingHeaderReader> routing;
    std::optional<FragmentHeaderReader> fragment;
    std::optional<AuthenticationHeaderReader> auth_header;
    std::optional<OptionsHeaderReader> destination_1st;
    std::optional<OptionsHeaderReader> destination_2nd;
    size_t total_headers_len = 0;
    uint8_t final_next_header = 0;
};

namespace detail {
// A chain from its slot bits (flags >> shift) and zp_ext_offsets entries;
// the offsets are relative to the IPv6 payload at frame[payload_off..].
inline ExtensionHeaders ext_headers(Bytes frame, size_t payload_off, uint32_t flags, int shift,
                                    const uint16_t* off, size_t total, uint8_t final_nh) {
    ExtensionHeaders eh;
    auto at = [&](int k) { return frame.sub(payload_off + off[k]); };
    if (flags & (1u << (shift + ZP_EXT_HBH))) eh.hop_by_hop.emplace(at(ZP_EXT_HBH));
    if (flags & (1u << (shift + ZP_EXT_RT))) eh.routing.emplace(at(ZP_EXT_RT));
    if (flags & (1u << (shift + ZP_EXT_FRAG))) eh.fragment.emplace(at(ZP_EXT_FRAG));
    if (flags & (1u << (shift + ZP_EXT_AH))) eh.auth_header.emplace(at(ZP_EXT_AH));
    if (flags & (1u << (shift + ZP_EXT_DST1))) eh.destination_1st.emplace(at(ZP_EXT_DST1));
    if (flags & (1u << (shift + ZP_EXT_DST2))) eh.destination_2nd.emplace(at(ZP_EXT_DST2));
    eh.total_headers_len = total;
    eh.final_next_header = final_nh;
    return eh;
}
}  // namespace detail

// ipv6.rs:135-286
class IPv6Reader : public detail::Checked<IPv6Reader, ZP_READER_IPV6> {
public:
    Bytes bytes;
    std::optional<ExtensionHeaders> extension_headers;
    size_t extension_headers_len = 0;
    explicit IPv6Reader(Bytes b) : bytes(b) {}
    // ipv6.rs:147-167: the constructor runs the extension walk (ipv6.rs:159)
    static IPv6Reader from_info(Bytes b, const zp_reader_info& i) {
        IPv6Reader r(b);
        if (i.flags & ZP_F_EXT) {
            r.extension_headers = detail::ext_headers(b, 40, i.flags, 12, i.ext.off, i.ext.len,
                                                      i.final_nh);
            r.extension_headers_len = i.ext.len;
        }
        return r;
    }
    uint8_t version() const { return bytes[0] >> 4; }
    uint8_t traffic_class() const { return (uint8_t)(((bytes[0] & 0x0F) << 4) | (bytes[1] >> 4)); }
    uint32_t flow_label() const {
        return ((uint32_t)(bytes[1] & 0x0F) << 16) | ((uint32_t)bytes[2] << 8) | bytes[3];
    }
    uint16_t payload_length() const { return detail::be16(bytes, 4); }
    uint8_t next_header() const { return bytes[6]; }
    uint8_t final_next_header() const {   // ipv6.rs:219-227
        return extension_headers ? extension_headers->final_next_header : next_header();
    }
    uint8_t hop_limit() const { return bytes[7]; }
    std::array<uint8_t, 16> src_addr() const { return detail::arr<16>(bytes, 8); }
    std::array<uint8_t, 16> dest_addr() const { return detail::arr<16>(bytes, 24); }
    size_t header_len() const { return 40; }
    Bytes header() const { return bytes.sub(0, 40); }
    Bytes payload() const { return bytes.sub(40); }
    Bytes upper_layer_payload() const { return bytes.sub(40 + extension_headers_len); }
};

// tcp.rs:132-244
class TcpReader : public detail::Checked<TcpReader, ZP_READER_TCP> {
public:
    Bytes bytes;
    explicit TcpReader(Bytes b) : bytes(b) {}
    uint16_t src_port() const { return detail::be16(bytes, 0); }
    uint16_t dest_port() const { return detail::be16(bytes, 2); }
    uint32_t sequence_number() const { return detail::be32(bytes, 4); }
    uint32_t ack_number() const { return detail::be32(bytes, 8); }
    uint8_t data_offset() const { return bytes[12] >> 4; }
    uint8_t reserved() const { return bytes[12] & 0x0F; }
    uint8_t flags() const { return bytes[13]; }
    uint16_t window_size() const { return detail::be16(bytes, 14); }
    uint16_t checksum() const { return detail::be16(bytes, 16); }
    uint16_t urgent_pointer() const { return detail::be16(bytes, 18); }
    size_t header_len() const { return (size_t)data_offset() * 4; }
    Bytes header() const { check(); return bytes.sub(0, header_len()); }   // tcp.rs:223-231
    Bytes payload() const { check(); return bytes.sub(header_len()); }     // tcp.rs:235-243
private:
    void check() const {
        if (header_len() > bytes.size()) detail::fail(ZP_ERR_TCP_HDR_EXCEEDS);
    }
};

// udp.rs:94-154
class UdpReader : public detail::Checked<UdpReader, ZP_READER_UDP> {
public:
    Bytes bytes;
    explicit UdpReader(Bytes b) : bytes(b) {}
    uint16_t src_port() const { return detail::be16(bytes, 0); }
    uint16_t dest_port() const { return detail::be16(bytes, 2); }
    uint16_t length() const { return detail::be16(bytes, 4); }
    uint16_t checksum() const { return detail::be16(bytes, 6); }
    size_t header_len() const { return 8; }
    Bytes header() const { return bytes.sub(0, 8); }
    Bytes payload() const { return bytes.sub(8); }
};

// icmpv4.rs:83-135 / icmpv6.rs:80-132
class IcmpReader {
public:
    Bytes bytes;
    explicit IcmpReader(Bytes b) : bytes(b) {}
    uint8_t icmp_type() const { return bytes[0]; }
    uint8_t icmp_code() const { return bytes[1]; }
    uint16_t checksum() const { return detail::be16(bytes, 2); }
    size_t header_len() const { return 8; }
    Bytes header() const { return bytes.sub(0, 8); }
    Bytes payload() const { return bytes.sub(8); }
};
class Icmpv4Reader : public IcmpReader, public detail::Checked<Icmpv4Reader, ZP_READER_ICMPV4> {
public:
    using IcmpReader::IcmpReader;
};
class Icmpv6Reader : public IcmpReader, public detail::Checked<Icmpv6Reader, ZP_READER_ICMPV6> {
public:
    using IcmpReader::IcmpReader;
};

// misc.rs:6-9: IpInIp::Ipv4(IPv4Reader) | IpInIp::Ipv6(IPv6Reader)
struct IpInIp {
    enum class Kind { Ipv4, Ipv6 } kind;
    std::optional<IPv4Reader> ipv4;
    std::optional<IPv6Reader> ipv6;
};

// parser.rs:22-32
struct PacketParser {
    std::optional<EthernetReader> ethernet;
    std::optional<ArpReader> arp;
    std::optional<IPv4Reader> ipv4;
    std::optional<IPv6Reader> ipv6;
    std::optional<IpInIp> ip_in_ip;
    std::optional<TcpReader> tcp;
    std::optional<UdpReader> udp;
    std::optional<Icmpv4Reader> icmpv4;
    std::optional<Icmpv6Reader> icmpv6;

    // Rebuilds the parse result of `frame` from its record (no re-parse).
    // outer / inner: the frame's zp_ext_offsets entries (ext[i], ext[n + i]
    // of the batch), needed when the record flags that chain.
    // Throws zp::Error when the record holds an error (the reference's Err).
    static PacketParser from_record(Bytes frame, const zp_record& r,
                                    const zp_ext_offsets* outer = nullptr,
                                    const zp_ext_offsets* inner = nullptr) {
        if (zp_rec_err(r)) detail::fail((int)zp_rec_err(r));
        const uint32_t flags = r.flags & ZP_F_MASK;
        zp_ext_offsets inl{};
        if (zp_rec_chain_inline(r)) {                 // ABI v6: the outer chain in the record
            zp_rec_chain(r, &inl);
            outer = &inl;
        }
        if (((flags & ZP_F_EXT) && !outer) || ((flags & ZP_F_INNER_EXT) && !inner))
            throw std::invalid_argument("from_record: the record flags an extension chain");
        PacketParser p;
        // both record forms: the far-L4 one (ABI v5) reads the Ethernet header
        // length and the ip_in_ip offset from the frame (zp_rec_decode)
        size_t hl = zp_rec_eth_len(r), io = zp_rec_inner_off(r);
        if (zp_rec_is_far(r)) {
            // (zp_rec_decode restated, header-only) ethernet.rs:155-179, then
            // the ip_in_ip header behind the outer IP header
            if (!(flags & ZP_F_IP_IN_IP))
                throw std::invalid_argument("from_record: far-L4 record without ip_in_ip");
            // the offsets the record implies must lie in the frame (as zp_rec_decode checks)
            if (zp_rec_l4_off(r) >= frame.len || frame.len < 14)
                throw std::invalid_argument("from_record: frame too short for the record");
            const uint32_t t = detail::be16(frame, 12);
            hl = t == 0x8100 ? 18 : t == 0x88A8 ? 22 : 14;
            if (hl >= frame.len)
                throw std::invalid_argument("from_record: frame too short for the record");
            io = (flags & ZP_F_IPV6) ? hl + 40 + ((flags & ZP_F_EXT) ? outer->len : 0)
                                     : hl + (frame[hl] & 15u) * 4;   // ipv4.rs:228-258
            if (io >= frame.len)
                throw std::invalid_argument("from_record: frame too short for the record");
        }
        if (flags & ZP_F_ETHERNET) p.ethernet.emplace(frame, hl);
        if (flags & ZP_F_ARP) p.arp.emplace(frame.sub(hl));
        if (flags & ZP_F_IPV4) p.ipv4.emplace(frame.sub(hl));
        if (flags & ZP_F_IPV6) {
            IPv6Reader v6(frame.sub(hl));
            if (flags & ZP_F_EXT) {
                v6.extension_headers = detail::ext_headers(frame, hl + 40, flags, 12, outer->off,
                                                           outer->len, outer->final_nh);
                v6.extension_headers_len = outer->len;
            }
            p.ipv6 = v6;
        }
        if (flags & ZP_F_IP_IN_IP) {
            IpInIp ii;
            if (flags & ZP_F_IP_IN_IP_V6) {
                ii.kind = IpInIp::Kind::Ipv6;
                IPv6Reader v6(frame.sub(io));
                if (flags & ZP_F_INNER_EXT) {
                    v6.extension_headers = detail::ext_headers(frame, io + 40, flags, 18,
                                                               inner->off, inner->len,
                                                               inner->final_nh);
                    v6.extension_headers_len = inner->len;
                }
                ii.ipv6 = v6;
            } else {
                ii.kind = IpInIp::Kind::Ipv4;
                ii.ipv4.emplace(frame.sub(io));
            }
            p.ip_in_ip = ii;
        }
        const Bytes l4 = frame.sub(zp_rec_l4_off(r));
        if (flags & ZP_F_TCP) p.tcp.emplace(l4);
        if (flags & ZP_F_UDP) p.udp.emplace(l4);
        if (flags & ZP_F_ICMPV4) p.icmpv4.emplace(l4);
        if (flags & ZP_F_ICMPV6) p.icmpv6.emplace(l4);
        return p;
    }

    // PacketParser::parse (parser.rs:53) for one frame, through the GPU path
    // (zp_parse_one on `ctx`). Throws zp::Error on a parse error and
    // std::runtime_error on a HIP failure.
    // ext_out (optional, 2 entries) receives the outer and ip_in_ip chains.
    static PacketParser parse(zp_ctx* ctx, Bytes frame, zp_ext_offsets* ext_out = nullptr) {
        zp_record r{};
        zp_ext_offsets e[2] = {};
        const int rc = zp_parse_one(ctx, frame.ptr, frame.len, &r, e);
        if (rc < 0) throw std::runtime_error(std::string("zp_parse_one: ") + zp_last_error());
        if (ext_out) { ext_out[0] = e[0]; ext_out[1] = e[1]; }
        return from_record(frame, r, &e[0], &e[1]);
    }
};

// RAII owner of a zp_ctx (host-memory batches, single frames).
class Context {
public:
    explicit Context(int device = 0, uint64_t chunk_bytes = 0)
        : ctx_(zp_ctx_create(device, chunk_bytes)) {
        if (!ctx_) throw std::runtime_error(std::string("zp_ctx_create: ") + zp_last_error());
    }
    ~Context() { zp_ctx_destroy(ctx_); }
    // zp_parse_one's mode: idle_us > 0 = the device's resident server (the
    // default), 0 = one launch per call; stops the device's server.
    void parse_one_mode(uint32_t idle_us) { zp_parse_one_config(ctx_, idle_us); }
    Context(const Context&) = delete;
    Context& operator=(const Context&) = delete;
    zp_ctx* get() const { return ctx_; }

    // n frames of a host buffer -> host records (H2D, parse, D2H); ext:
    // nullptr or 2n entries (zero_packet.h, zp_ext_offsets).
    void parse_batch(const uint8_t* arena, uint64_t arena_bytes, const uint64_t* offs,
                     const uint32_t* lens, uint64_t n, zp_record* records,
                     zp_ext_offsets* ext = nullptr) {
        if (zp_parse_batch_host(ctx_, arena, arena_bytes, offs, lens, n, records, ext) < 0)
            throw std::runtime_error(std::string("zp_parse_batch_host: ") + zp_last_error());
    }
    PacketParser parse(Bytes frame, zp_ext_offsets* ext_out = nullptr) {
        return PacketParser::parse(ctx_, frame, ext_out);
    }
private:
    zp_ctx* ctx_;
};

// The per-frame drop-in, `zp::parse(frame)` where the reference has
// `PacketParser::parse(frame)` (parser.rs:53): one small Context per thread
// and device, created on first use (zp_device_current), so threads parse
// concurrently through the device's shared resident server (INTEGRATION.md
// §1.2). Frames over 64 KiB take the context's batch path; its 1 MiB chunk
// refuses longer ones (use a Context with a larger chunk for jumbo traffic).
inline PacketParser parse(Bytes frame, zp_ext_offsets* ext_out = nullptr) {
    struct PerDevice {
        std::unique_ptr<Context> c[64];
    };
    thread_local PerDevice mine;
    const int dev = zp_device_current();
    if (dev < 0 || dev >= 64) throw std::runtime_error(std::string("zp_device_current: ") + zp_last_error());
    if (!mine.c[dev]) mine.c[dev] = std::make_unique<Context>(dev, 1ull << 20);
    return mine.c[dev]->parse(frame, ext_out);
}

// A host batch over several devices (one Context each): byte-balanced
// contiguous ranges, concurrently (zp_parse_batch_host_multi).
inline void parse_batch_multi(Context* const* ctxs, int nctx, const uint8_t* arena,
                              uint64_t arena_bytes, const uint64_t* offs, const uint32_t* lens,
                              uint64_t n, zp_record* records, zp_ext_offsets* ext = nullptr) {
    zp_ctx* raw[64];
    if (nctx < 1 || nctx > 64) throw std::invalid_argument("parse_batch_multi: 1..64 contexts");
    for (int d = 0; d < nctx; ++d) raw[d] = ctxs[d]->get();
    if (zp_parse_batch_host_multi(raw, nctx, arena, arena_bytes, offs, lens, n, records,
                                  ext) < 0)
        throw std::runtime_error(std::string("zp_parse_batch_host_multi: ") + zp_last_error());
}

// Device-resident batch (the hot path): enqueue on a hipStream_t (void*).
inline void parse_batch_device(const uint8_t* arena, const uint64_t* offs, const uint32_t* lens,
                               uint64_t n, zp_record* records, zp_ext_offsets* ext,
                               void* stream) {
    if (zp_parse_batch_device(arena, offs, lens, n, records, ext, stream) < 0)
        throw std::runtime_error(std::string("zp_parse_batch_device: ") + zp_last_error());
}


// Per-batch counters (zp_stats_device): adds into counts[ZP_STATS_COUNT].
inline void stats_device(const zp_record* records, uint64_t n, uint64_t* counts, void* stream) {
    if (zp_stats_device(records, n, counts, stream) < 0)
        throw std::runtime_error(std::string("zp_stats_device: ") + zp_last_error());
}

// ---------------------------------------------------------------------------
// Host-ring ingestion: RAII over zp_ring_*.
// ---------------------------------------------------------------------------
class Ring {
public:
    Ring(int device, uint32_t nslots, uint64_t slot_bytes, uint64_t slot_frames)
        : r_(zp_ring_create(device, nslots, slot_bytes, slot_frames)) {
        if (!r_) throw std::runtime_error(std::string("zp_ring_create: ") + zp_last_error());
    }
    ~Ring() { zp_ring_destroy(r_); }
    Ring(const Ring&) = delete;
    Ring& operator=(const Ring&) = delete;
    // The next FREE slot (pinned host views), or std::nullopt on timeout.
    std::optional<zp_ring_slot> acquire(int64_t timeout_ms = -1) {
        zp_ring_slot s{};
        const int rc = zp_ring_acquire(r_, &s, timeout_ms);
        if (rc == ZP_RING_TIMEOUT) return std::nullopt;
        check(rc, "zp_ring_acquire");
        return s;
    }
    void submit(const zp_ring_slot& s, uint64_t n) { check(zp_ring_submit(r_, s.id, n), "zp_ring_submit"); }
    // The oldest submitted slot with its records, or std::nullopt on timeout.
    std::optional<zp_ring_slot> wait(int64_t timeout_ms = -1) {
        zp_ring_slot s{};
        const int rc = zp_ring_wait(r_, &s, timeout_ms);
        if (rc == ZP_RING_TIMEOUT) return std::nullopt;
        check(rc, "zp_ring_wait");
        return s;
    }
    void release(const zp_ring_slot& s) { check(zp_ring_release(r_, s.id), "zp_ring_release"); }

private:
    static void check(int rc, const char* what) {
        if (rc < 0) throw std::runtime_error(std::string(what) + ": " + zp_last_error());
    }
    zp_ring* r_;
};

// ---------------------------------------------------------------------------
// Batched PacketBuilder. Mirrors builder.rs:55-909:
// the same method names and argument order, and the typestate graph of
// builder.rs:817-909 is checked at compile time (a method a state does not
// have fails a static_assert, as the Rust chain fails to compile). The chain
// is recorded and runs on the GPU at build(), which throws zp::BuildError
// with the reference's message when a step returns Err.
// ---------------------------------------------------------------------------
class BuildError : public std::runtime_error {
public:
    BuildError(int code, size_t header_len)
        : std::runtime_error(zp_build_err_str(code) ? zp_build_err_str(code) : "build error"),
          code_(code), header_len_(header_len) {}
    int code() const { return code_; }
    size_t header_len() const { return header_len_; }
private:
    int code_;
    size_t header_len_;
};

namespace bstate {   // builder.rs:29-45
enum S { Raw, Eth, Arp, V4, V6, Hbh, D1, Rt, Fr, Ah, D2, V4e, V6e, L4, Bad };
constexpr int next(int st, int k) {
    const bool l4v4 = k == ZP_B_TCP || k == ZP_B_UDP || k == ZP_B_ICMPV4;
    const bool l4v6 = k == ZP_B_TCP || k == ZP_B_UDP || k == ZP_B_ICMPV6;
    if (st == Raw) return (k >= ZP_B_ETHERNET && k <= ZP_B_ETHERNET_QINQ) ? Eth : Bad;
    if (st == Eth) return k == ZP_B_ARP ? Arp : k == ZP_B_IPV4 ? V4 : k == ZP_B_IPV6 ? V6 : Bad;
    if (st == V4) return l4v4 ? L4 : k == ZP_B_IPV4 ? V4e : k == ZP_B_IPV6 ? V6e : Bad;
    if (st == V4e) return l4v4 ? L4 : Bad;
    if (st == V6e) return l4v6 ? L4 : Bad;
    if (st >= V6 && st <= D2) {
        if (l4v6) return L4;
        if (k == ZP_B_IPV4) return V4e;
        if (k == ZP_B_IPV6) return V6e;
        const int e = k == ZP_B_HOP_BY_HOP ? 0 : k == ZP_B_DEST_OPTS1 ? 1 : k == ZP_B_ROUTING ? 2
                    : k == ZP_B_FRAGMENT ? 3 : k == ZP_B_AUTH ? 4 : k == ZP_B_DEST_OPTS2 ? 5 : -1;
        const int succ[7] = {0x3F, 0x3E, 0x04, 0x38, 0x30, 0x20, 0x00};
        return (e >= 0 && ((succ[st - V6] >> e) & 1)) ? Hbh + e : Bad;
    }
    return Bad;
}
}  // namespace bstate

template <int S = bstate::Raw>
class PacketBuilder {
public:
    // PacketBuilder::new (builder.rs:98): the caller's buffer, built in place.
    PacketBuilder(uint8_t* bytes, size_t len) : bytes_(bytes), len_(len) {}

    // The address type of tcp/udp: &[u8; 4] under IPv4 states, else &[u8; 16].
    using Addr = std::conditional_t<S == bstate::V4 || S == bstate::V4e,
                                    std::array<uint8_t, 4>, std::array<uint8_t, 16>>;
    using Mac = std::array<uint8_t, 6>;
    using Ip4 = std::array<uint8_t, 4>;
    using Ip6 = std::array<uint8_t, 16>;

    auto ethernet(const Mac& src_mac, const Mac& dest_mac, uint16_t ethertype) {
        return push<ZP_B_ETHERNET>([&](zp_build_op& o) {
            cp(o.src, src_mac); cp(o.dst, dest_mac); o.h[0] = ethertype; });
    }
    auto ethernet_vlan(const Mac& src_mac, const Mac& dest_mac, uint16_t ethertype, uint16_t tci) {
        return push<ZP_B_ETHERNET_VLAN>([&](zp_build_op& o) {
            cp(o.src, src_mac); cp(o.dst, dest_mac); o.h[0] = ethertype; o.h[1] = tci; });
    }
    auto ethernet_qinq(const Mac& src_mac, const Mac& dest_mac, uint16_t ethertype, uint16_t tci1,
                       uint16_t tci2) {
        return push<ZP_B_ETHERNET_QINQ>([&](zp_build_op& o) {
            cp(o.src, src_mac); cp(o.dst, dest_mac);
            o.h[0] = ethertype; o.h[1] = tci1; o.h[2] = tci2; });
    }
    auto arp(uint16_t hardware_type, uint16_t protocol_type, uint8_t hardware_address_length,
             uint8_t protocol_address_length, uint16_t operation, const Mac& src_mac,
             const Ip4& src_ip, const Mac& dest_mac, const Ip4& dest_ip) {
        return push<ZP_B_ARP>([&](zp_build_op& o) {
            o.h[0] = hardware_type; o.h[1] = protocol_type; o.h[2] = operation;
            o.b[0] = hardware_address_length; o.b[1] = protocol_address_length;
            cp(o.src, src_mac); cp(o.src + 6, src_ip); cp(o.dst, dest_mac); cp(o.dst + 6, dest_ip); });
    }
    auto ipv4(uint8_t version, uint8_t ihl, uint8_t dscp, uint8_t ecn, uint16_t total_length,
              uint16_t identification, uint8_t flags, uint16_t fragment_offset, uint8_t ttl,
              uint8_t protocol, const Ip4& src_ip, const Ip4& dest_ip) {
        return push<ZP_B_IPV4>([&](zp_build_op& o) {
            o.b[0] = version; o.b[1] = ihl; o.b[2] = dscp; o.b[3] = ecn; o.b[4] = flags;
            o.b[5] = ttl; o.b[6] = protocol; o.h[0] = total_length; o.h[1] = identification;
            o.h[2] = fragment_offset; cp(o.src, src_ip); cp(o.dst, dest_ip); });
    }
    auto ipv6(uint8_t version, uint8_t traffic_class, uint32_t flow_label, uint16_t payload_length,
              uint8_t next_header, uint8_t hop_limit, const Ip6& src_addr, const Ip6& dest_addr) {
        return push<ZP_B_IPV6>([&](zp_build_op& o) {
            o.b[0] = version; o.b[1] = traffic_class; o.b[2] = next_header; o.b[3] = hop_limit;
            o.w[0] = flow_label; o.h[0] = payload_length; cp(o.src, src_addr); cp(o.dst, dest_addr); });
    }
    auto hop_by_hop(uint8_t next_header, uint8_t extension_len, Bytes options) {
        return push<ZP_B_HOP_BY_HOP>([&](zp_build_op& o) {
            o.b[0] = next_header; o.b[1] = extension_len; blob(o, options); });
    }
    auto destination_options1(uint8_t next_header, uint8_t extension_len, Bytes options) {
        return push<ZP_B_DEST_OPTS1>([&](zp_build_op& o) {
            o.b[0] = next_header; o.b[1] = extension_len; blob(o, options); });
    }
    auto routing_header(uint8_t next_header, uint8_t header_ext_len, uint8_t routing_type,
                        uint8_t segments_left, Bytes data) {
        return push<ZP_B_ROUTING>([&](zp_build_op& o) {
            o.b[0] = next_header; o.b[1] = header_ext_len; o.b[2] = routing_type;
            o.b[3] = segments_left; blob(o, data); });
    }
    auto fragment_header(uint8_t next_header, uint16_t fragment_offset, bool m_flag,
                         uint32_t identification) {
        return push<ZP_B_FRAGMENT>([&](zp_build_op& o) {
            o.b[0] = next_header; o.h[0] = fragment_offset; o.b[1] = m_flag ? 1 : 0;
            o.w[0] = identification; });
    }
    auto authentication_header(uint8_t next_header, uint8_t payload_len, uint32_t spi,
                               uint32_t seq_num, Bytes auth_data) {
        return push<ZP_B_AUTH>([&](zp_build_op& o) {
            o.b[0] = next_header; o.b[1] = payload_len; o.w[0] = spi; o.w[1] = seq_num;
            blob(o, auth_data); });
    }
    auto destination_options2(uint8_t next_header, uint8_t extension_len, Bytes options) {
        return push<ZP_B_DEST_OPTS2>([&](zp_build_op& o) {
            o.b[0] = next_header; o.b[1] = extension_len; blob(o, options); });
    }
    auto tcp(const Addr& src_ip, uint16_t src_port, const Addr& dest_ip, uint16_t dest_port,
             uint32_t sequence_number, uint32_t acknowledgment_number, uint8_t data_offset,
             uint8_t reserved, uint8_t flags, uint16_t window_size, uint16_t urgent_pointer,
             std::optional<Bytes> payload = std::nullopt) {
        return push<ZP_B_TCP>([&](zp_build_op& o) {
            cp(o.src, src_ip); cp(o.dst, dest_ip); o.h[0] = src_port; o.h[1] = dest_port;
            o.w[0] = sequence_number; o.w[1] = acknowledgment_number; o.b[0] = data_offset;
            o.b[1] = reserved; o.b[2] = flags; o.h[2] = window_size; o.h[3] = urgent_pointer;
            opt_blob(o, payload); });
    }
    auto udp(const Addr& src_addr, uint16_t src_port, const Addr& dest_addr, uint16_t dest_port,
             uint16_t length, std::optional<Bytes> payload = std::nullopt) {
        return push<ZP_B_UDP>([&](zp_build_op& o) {
            cp(o.src, src_addr); cp(o.dst, dest_addr); o.h[0] = src_port; o.h[1] = dest_port;
            o.h[2] = length; opt_blob(o, payload); });
    }
    auto icmpv4(uint8_t icmp_type, uint8_t icmp_code, std::optional<Bytes> payload = std::nullopt) {
        return push<ZP_B_ICMPV4>([&](zp_build_op& o) {
            o.b[0] = icmp_type; o.b[1] = icmp_code; opt_blob(o, payload); });
    }
    auto icmpv6(const Ip6& src_addr, const Ip6& dest_addr, uint8_t icmp_type, uint8_t icmp_code,
                std::optional<Bytes> payload = std::nullopt) {
        return push<ZP_B_ICMPV6>([&](zp_build_op& o) {
            cp(o.src, src_addr); cp(o.dst, dest_addr); o.b[0] = icmp_type; o.b[1] = icmp_code;
            opt_blob(o, payload); });
    }

    // PacketBuilder::build (builder.rs:87): runs the chain on the GPU through
    // ctx and returns the buffer. Throws BuildError on a step's Err.
    Bytes build(zp_ctx* ctx) {
        const uint64_t off = 0;
        const uint32_t n = (uint32_t)len_;
        const uint32_t start[2] = {0, (uint32_t)ops_.size()};
        zp_build_result r{};
        const int rc = zp_build_batch_host(ctx, bytes_, len_, &off, &n, 1,
                                           ops_.empty() ? nullptr : ops_.data(), start,
                                           data_.empty() ? nullptr : data_.data(), data_.size(), &r);
        if (rc < 0) throw std::runtime_error(std::string("zp_build_batch_host: ") + zp_last_error());
        header_len_ = r.header_len;
        if (r.err) throw BuildError(r.err, r.header_len);
        return Bytes{bytes_, len_};
    }
    // builder.rs:65-84, valid after build()
    size_t header_len() const { return header_len_; }
    size_t payload_len() const { return len_ - header_len_; }
    Bytes payload() const { return Bytes{bytes_ + header_len_, len_ - header_len_}; }

    const std::vector<zp_build_op>& ops() const { return ops_; }
    const std::vector<uint8_t>& data() const { return data_; }

private:
    template <int> friend class PacketBuilder;
    template <size_t N>
    static void cp(uint8_t* d, const std::array<uint8_t, N>& a) { std::memcpy(d, a.data(), N); }
    void blob(zp_build_op& o, Bytes b) {
        o.data_off = (uint32_t)data_.size();
        o.data_len = (uint32_t)b.len;
        data_.insert(data_.end(), b.ptr, b.ptr + b.len);
    }
    void opt_blob(zp_build_op& o, const std::optional<Bytes>& b) {
        if (b) blob(o, *b);
        else { o.data_off = 0; o.data_len = ZP_BUILD_NO_DATA; }
    }
    template <int K, class F>
    PacketBuilder<bstate::next(S, K)> push(F&& fill) {
        static_assert(bstate::next(S, K) != bstate::Bad,
                      "this PacketBuilder state has no such method (builder.rs:817-909)");
        zp_build_op o{};
        o.kind = (uint8_t)K;
        fill(o);
        ops_.push_back(o);
        PacketBuilder<bstate::next(S, K)> nb(bytes_, len_);
        nb.ops_ = std::move(ops_);
        nb.data_ = std::move(data_);
        return nb;
    }
    uint8_t* bytes_;
    size_t len_;
    size_t header_len_ = 0;
    std::vector<zp_build_op> ops_;
    std::vector<uint8_t> data_;
};

}  // namespace zp

#endif  // ZERO_PACKET_HPP
