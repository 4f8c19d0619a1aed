// Test driver for the checked reader constructors of include/zero_packet.hpp
// (XReader::create / try_create = the reference's XReader::new, README.md:
// 110-115) and the checksum primitives. stdin lines:
//   r <kind> <slice hex>          -> one summary line (tests/test_readers.py
//                                    builds the same line from the Python facade)
//   cs <acc> <data hex>           -> "<internet_checksum> <verify>"
//   ph <proto> <len> <src> <dst>  -> "<pseudo_header>"
#include <cstdio>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "zero_packet.hpp"

static std::vector<uint8_t> unhex(const std::string& s) {
    std::vector<uint8_t> v(s.size() / 2);
    for (size_t i = 0; i < v.size(); ++i) v[i] = (uint8_t)std::stoul(s.substr(2 * i, 2), nullptr, 16);
    return v;
}

// "<len>" of an accessor's slice, "e<code>" on zp::Error, "panic" where the
// reference would panic (std::out_of_range here).
template <class F>
static std::string len_of(F&& f) {
    try {
        return std::to_string(f().size());
    } catch (const zp::Error& e) {
        return "e" + std::to_string(e.code());
    } catch (const std::out_of_range&) {
        return "panic";
    }
}

static std::string ext_summary(const zp::IPv6Reader& r) {
    std::ostringstream o;
    o << " fnh=" << (int)r.final_next_header() << " ulp=" << r.upper_layer_payload().size();
    if (!r.extension_headers) return o.str() + " ext=-";
    const auto& e = *r.extension_headers;
    o << " ext=" << e.total_headers_len << "," << (int)e.final_next_header;
    auto slot = [&](const char* n, const zp::Bytes* b) {
        if (b) o << "," << n << "@" << (r.bytes.size() - b->size());
    };
    slot("hbh", e.hop_by_hop ? &e.hop_by_hop->bytes : nullptr);
    slot("rt", e.routing ? &e.routing->bytes : nullptr);
    slot("frag", e.fragment ? &e.fragment->bytes : nullptr);
    slot("ah", e.auth_header ? &e.auth_header->bytes : nullptr);
    slot("d1", e.destination_1st ? &e.destination_1st->bytes : nullptr);
    slot("d2", e.destination_2nd ? &e.destination_2nd->bytes : nullptr);
    return o.str();
}

static std::string reader_line(int kind, zp::Bytes b) {
    std::ostringstream o;
    try {
        o << "ok";
        switch (kind) {
        case ZP_READER_ETHERNET: {
            const auto r = zp::EthernetReader::create(b);
            o << " hl=" << r.header_len() << " et=" << r.ethertype() << " vlan=";
            if (auto t = r.vlan_tag()) o << t->second; else o << "-";
            break;
        }
        case ZP_READER_ARP: o << " oper=" << zp::ArpReader::create(b).oper(); break;
        case ZP_READER_IPV4: {
            const auto r = zp::IPv4Reader::create(b);
            o << " hl=" << r.header_len() << " vc=";
            try { o << (r.valid_checksum() ? 1 : 0); } catch (const zp::Error& e) { o << "e" << e.code(); }
            o << " p=" << len_of([&] { return r.payload(); });
            break;
        }
        case ZP_READER_IPV6: o << ext_summary(zp::IPv6Reader::create(b)); break;
        case ZP_READER_OPTIONS: {
            const auto r = zp::OptionsHeaderReader::create(b);
            o << " hl=" << r.header_len() << " opt=" << len_of([&] { return r.options(); })
              << " p=" << len_of([&] { return r.payload(); });
            break;
        }
        case ZP_READER_ROUTING: {
            const auto r = zp::RoutingHeaderReader::create(b);
            o << " hl=" << r.header_len() << " data=" << len_of([&] { return r.data(); })
              << " p=" << len_of([&] { return r.payload(); });
            break;
        }
        case ZP_READER_FRAGMENT: {
            const auto r = zp::FragmentHeaderReader::create(b);
            o << " fo=" << r.fragment_offset() << " m=" << (r.m_flag() ? 1 : 0)
              << " id=" << r.identification();
            break;
        }
        case ZP_READER_AUTH: {
            const auto r = zp::AuthenticationHeaderReader::create(b);
            o << " hl=" << r.header_len() << " ad=" << len_of([&] { return r.authentication_data(); })
              << " p=" << len_of([&] { return r.payload(); });
            break;
        }
        case ZP_READER_TCP: {
            const auto r = zp::TcpReader::create(b);
            o << " hl=" << r.header_len() << " h=" << len_of([&] { return r.header(); })
              << " p=" << len_of([&] { return r.payload(); });
            break;
        }
        case ZP_READER_UDP: {
            const auto r = zp::UdpReader::create(b);
            o << " len=" << r.length() << " p=" << r.payload().size();
            break;
        }
        case ZP_READER_ICMPV4: {
            const auto r = zp::Icmpv4Reader::create(b);
            o << " t=" << (int)r.icmp_type() << " c=" << (int)r.icmp_code();
            break;
        }
        case ZP_READER_ICMPV6: {
            const auto r = zp::Icmpv6Reader::create(b);
            o << " t=" << (int)r.icmp_type() << " c=" << (int)r.icmp_code();
            break;
        }
        default: return "bad kind";
        }
    } catch (const zp::Error& e) {
        // try_create must agree with create
        int code = -1;
        bool none = false;
        switch (kind) {
        case ZP_READER_TCP: none = !zp::TcpReader::try_create(b, &code); break;
        case ZP_READER_IPV6: none = !zp::IPv6Reader::try_create(b, &code); break;
        default: none = true; code = e.code();
        }
        if (!none || code != e.code()) return "try_create disagrees";
        return "err=" + std::to_string(e.code()) + "|" + e.what();
    }
    return o.str();
}

int main() {
    std::string line;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string mode;
        in >> mode;
        if (mode == "r") {
            int kind;
            std::string hex;
            in >> kind >> hex;
            const std::vector<uint8_t> v = unhex(hex);
            std::cout << reader_line(kind, zp::Bytes{v.data(), v.size()}) << "\n";
        } else if (mode == "cs") {
            uint32_t acc;
            std::string hex;
            in >> acc >> hex;
            const std::vector<uint8_t> v = unhex(hex);
            const zp::Bytes b{v.data(), v.size()};
            std::cout << zp::internet_checksum(b, acc) << " " << zp::verify_internet_checksum(b, acc)
                      << "\n";
        } else if (mode == "ph") {
            int proto;
            size_t len;
            std::string sh, dh;
            in >> proto >> len >> sh >> dh;
            const std::vector<uint8_t> s = unhex(sh), d = unhex(dh);
            if (s.size() == 4) {
                std::array<uint8_t, 4> a, c;
                std::copy(s.begin(), s.end(), a.begin());
                std::copy(d.begin(), d.end(), c.begin());
                std::cout << zp::pseudo_header(a, c, (uint8_t)proto, len) << "\n";
            } else {
                std::array<uint8_t, 16> a, c;
                std::copy(s.begin(), s.end(), a.begin());
                std::copy(d.begin(), d.end(), c.begin());
                std::cout << zp::pseudo_header(a, c, (uint8_t)proto, len) << "\n";
            }
        }
    }
    return 0;
}
