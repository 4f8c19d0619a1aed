// Test driver for include/zero_packet.hpp (the C++ facade).
//   facade_main cpu   stdin lines "<frame hex> <zp_record hex> <2 x zp_ext_offsets hex>"
//                     -> PacketParser::from_record (no GPU, no library)
//   facade_main gpu   stdin lines "<frame hex>" -> PacketParser::parse through
//                     zp_parse_one (libzp_hip.so, the GPU path)
// One summary line per frame; tests/test_facade_cpp.py builds the same line
// from the Python facade and compares.
#include <cstdio>
#include <cstring>
#include <memory>
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

static void ext_summary(std::ostringstream& o, const std::optional<zp::ExtensionHeaders>& e) {
    if (!e) { o << ";ext=-"; return; }
    o << ";ext=" << e->total_headers_len << "," << (int)e->final_next_header;
    auto slot = [&](const char* n, bool present, size_t len) {
        if (present) o << "," << n << "@" << len;
    };
    slot("hbh", e->hop_by_hop.has_value(), e->hop_by_hop ? e->hop_by_hop->bytes.size() : 0);
    slot("rt", e->routing.has_value(), e->routing ? e->routing->bytes.size() : 0);
    slot("frag", e->fragment.has_value(), e->fragment ? e->fragment->bytes.size() : 0);
    slot("ah", e->auth_header.has_value(), e->auth_header ? e->auth_header->bytes.size() : 0);
    slot("d1", e->destination_1st.has_value(), e->destination_1st ? e->destination_1st->bytes.size() : 0);
    slot("d2", e->destination_2nd.has_value(), e->destination_2nd ? e->destination_2nd->bytes.size() : 0);
}

static void v6_summary(std::ostringstream& o, const zp::IPv6Reader& r) {
    o << r.bytes.size() << "," << (int)r.next_header() << "," << (int)r.final_next_header() << ","
      << r.extension_headers_len << "," << r.upper_layer_payload().size() << "," << r.flow_label();
    ext_summary(o, r.extension_headers);
}

static std::string summary(const zp::PacketParser& p) {
    std::ostringstream o;
    o << "ok";
    if (p.ethernet) {
        const auto& e = *p.ethernet;
        o << " eth:" << e.header_len() << "," << e.ethertype() << ",";
        if (auto t = e.vlan_tag()) o << t->first << "/" << t->second; else o << "-";
        o << ",";
        if (auto t = e.double_vlan_tag()) o << t->first.second << "/" << t->second.second; else o << "-";
    }
    if (p.arp) o << " arp:" << p.arp->oper() << "," << p.arp->htype() << "," << (int)p.arp->spa()[3];
    if (p.ipv4) o << " ipv4:" << p.ipv4->bytes.size() << "," << (int)p.ipv4->ihl() << ","
                  << p.ipv4->total_length() << "," << (int)p.ipv4->protocol() << ","
                  << p.ipv4->checksum() << "," << (int)p.ipv4->src_ip()[0];
    if (p.ipv6) { o << " ipv6:"; v6_summary(o, *p.ipv6); }
    if (p.ip_in_ip) {
        if (p.ip_in_ip->kind == zp::IpInIp::Kind::Ipv4)
            o << " iip4:" << p.ip_in_ip->ipv4->bytes.size() << "," << (int)p.ip_in_ip->ipv4->protocol();
        else { o << " iip6:"; v6_summary(o, *p.ip_in_ip->ipv6); }
    }
    if (p.tcp) o << " tcp:" << p.tcp->bytes.size() << "," << p.tcp->src_port() << ","
                 << p.tcp->dest_port() << "," << (int)p.tcp->data_offset() << "," << (int)p.tcp->flags();
    if (p.udp) o << " udp:" << p.udp->bytes.size() << "," << p.udp->src_port() << ","
                 << p.udp->dest_port() << "," << p.udp->length();
    if (p.icmpv4) o << " icmp4:" << p.icmpv4->bytes.size() << "," << (int)p.icmpv4->icmp_type() << ","
                    << (int)p.icmpv4->icmp_code();
    if (p.icmpv6) o << " icmp6:" << p.icmpv6->bytes.size() << "," << (int)p.icmpv6->icmp_type();
    return o.str();
}

int main(int argc, char** argv) {
    const bool gpu = argc > 1 && std::string(argv[1]) == "gpu";
#ifdef ZP_FACADE_GPU
    std::unique_ptr<zp::Context> ctx;
    if (gpu) ctx = std::make_unique<zp::Context>(0);
#else
    if (gpu) { std::fprintf(stderr, "built without ZP_FACADE_GPU\n"); return 2; }
#endif
    std::string line;
    [[maybe_unused]] uint64_t nline = 0;
    while (std::getline(std::cin, line)) {
        std::istringstream in(line);
        std::string fh, rh, eh;
        in >> fh >> rh >> eh;
        const std::vector<uint8_t> frame = unhex(fh);
        const zp::Bytes b{frame.data(), frame.size()};
        try {
            zp::PacketParser p;
            if (gpu) {
#ifdef ZP_FACADE_GPU
                // every other frame through the thread's implicit context
                p = (nline++ & 1) ? zp::parse(b) : ctx->parse(b);
#endif
            } else {
                zp_record r{};
                zp_ext_offsets e[2] = {};
                const auto rv = unhex(rh), ev = unhex(eh);
                std::memcpy(&r, rv.data(), sizeof r);
                std::memcpy(e, ev.data(), sizeof e);       // outer, ip_in_ip chain
                p = zp::PacketParser::from_record(b, r, &e[0], &e[1]);
            }
            std::cout << summary(p) << "\n";
        } catch (const zp::Error& e) {
            std::cout << "err=" << e.code() << "|" << e.what() << "\n";
        }
    }
    return 0;
}
