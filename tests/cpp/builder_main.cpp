// C++ facade tests for the §8(f) rows, written like the reference's own
// builder tests (builder.rs:911-1556): zp::PacketBuilder chains built on the
// GPU (zp_build_batch_host) and parsed back (zp_parse_one), and a zp::Ring
// round trip. Prints "<name> <hex>" for the byte-exact vectors (compared by
// tests/test_facade_cpp.py against the reference's should_be arrays) and
// "OK <name>" per passing check; exits non-zero on the first failure.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "zero_packet.hpp"

#define CHECK(c)                                                                  \
    do {                                                                          \
        if (!(c)) {                                                               \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);               \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

static void hex(const char* name, const uint8_t* p, size_t n) {
    std::printf("%s ", name);
    for (size_t i = 0; i < n; ++i) std::printf("%02x", p[i]);
    std::printf("\n");
}

using zp::PacketBuilder;
static const std::array<uint8_t, 6> M1{0x34, 0x97, 0xf6, 0x94, 0x02, 0x0f};
static const std::array<uint8_t, 6> M2{0x04, 0xb4, 0xfe, 0x9a, 0x81, 0xc7};
static const std::array<uint8_t, 4> IP1{192, 168, 1, 1}, IP2{192, 168, 1, 2};

int main() {
    zp::Context gpu(0);

    {   // builder.rs:919-993 write_payload
        uint8_t buffer[64] = {0};
        const uint8_t payload[10] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
        auto b = PacketBuilder<>(buffer, sizeof buffer)
                     .ethernet({1, 2, 3, 4, 5, 6}, {7, 8, 9, 10, 11, 12}, 0x0800)
                     .ipv4(4, 5, 0, 0, 50, 0, 0, 0, 64, 17, IP1, IP2)
                     .udp(IP1, 12345, IP2, 54321, 30, zp::Bytes{payload, 10});
        zp::Bytes packet = b.build(gpu.get());
        CHECK(b.header_len() == 14 + 20 + 8);
        const zp::Bytes pay = b.payload();
        CHECK(pay.len == 22);
        for (size_t i = 0; i < 22; ++i) CHECK(pay[i] == (i < 10 ? i + 1 : 0));
        zp::PacketParser p = gpu.parse(packet);
        CHECK(p.udp.has_value());
        CHECK(p.udp->payload().len == 22 && p.udp->payload()[9] == 10);
        std::printf("OK write_payload\n");
    }
    {   // builder.rs:995-1046 misc: header and payload lengths per state
        uint8_t packet[64] = {0};
        auto eth = PacketBuilder<>(packet, 64).ethernet(M1, {0xff, 0xff, 0xff, 0xff, 0xff, 0xff}, 2054);
        auto arp = eth.arp(1, 2048, 6, 4, 1, M1, IP1, {0, 0, 0, 0, 0, 0}, IP2);
        arp.build(gpu.get());
        CHECK(arp.header_len() == 14 + 28);
        CHECK(arp.payload_len() == 22);
        std::printf("OK misc\n");
    }
    {   // builder.rs:1048-1094 arp_in_ethernet
        uint8_t packet[42] = {0};
        PacketBuilder<>(packet, 42).ethernet(M1, {0xff, 0xff, 0xff, 0xff, 0xff, 0xff}, 2054)
            .arp(1, 2048, 6, 4, 1, M1, IP1, {0, 0, 0, 0, 0, 0}, IP2).build(gpu.get());
        hex("arp_in_ethernet", packet, 42);
    }
    {   // builder.rs:1096-1158 tcp_in_ipv4_in_ethernet
        uint8_t packet[54] = {0};
        PacketBuilder<>(packet, 54).ethernet(M1, M2, 2048)
            .ipv4(99, 5, 99, 123, 12345, 54321, 99, 12345, 123, 6, IP1, IP2)
            .tcp(IP1, 99, IP2, 11, 123, 321, 11, 99, 99, 4321, 1234).build(gpu.get());
        hex("tcp_in_ipv4_in_ethernet", packet, 54);
    }
    {   // builder.rs:1160-1209 udp_in_ipv4_in_ethernet
        uint8_t packet[54] = {0};
        PacketBuilder<>(packet, 54).ethernet(M1, M2, 2048)
            .ipv4(99, 5, 99, 123, 12345, 54321, 99, 12345, 123, 6, IP1, IP2)
            .udp(IP1, 99, IP2, 11, 4321).build(gpu.get());
        hex("udp_in_ipv4_in_ethernet", packet, 54);
    }
    {   // builder.rs:1211-1258 icmpv4_in_ipv4_in_ethernet
        uint8_t packet[64] = {0};
        PacketBuilder<>(packet, 64).ethernet(M1, M2, 2048)
            .ipv4(4, 5, 99, 123, 12345, 54321, 99, 12345, 123, 1, IP1, IP2)
            .icmpv4(8, 0).build(gpu.get());
        hex("icmpv4_in_ipv4_in_ethernet", packet, 64);
    }
    const std::array<uint8_t, 16> S6{0x20, 0x01, 0x0d, 0xb8, 0x85, 0xa3, 0, 0, 0, 0, 0x8a, 0x2e,
                                     0x03, 0x70, 0x73, 0x34};
    const std::array<uint8_t, 16> D6{0xfe, 0x80, 0, 0, 0, 0, 0, 0, 0x02, 0x02, 0xb3, 0xff,
                                     0xfe, 0x1e, 0x83, 0x29};
    {   // builder.rs:1260-1318 build_parse_ipv6
        uint8_t packet[64] = {0};
        PacketBuilder<>(packet, 64).ethernet(M1, M2, 34525).ipv6(6, 5, 4, 31, 17, 10, S6, D6)
            .udp(S6, 99, D6, 80, 10).build(gpu.get());
        hex("build_parse_ipv6", packet, 64);
        zp::PacketParser p = gpu.parse(zp::Bytes{packet, 64});
        CHECK(p.ethernet && p.ipv6 && p.udp && !p.arp && !p.icmpv4 && !p.tcp);
        std::printf("OK build_parse_ipv6\n");
    }
    {   // builder.rs:1450-1556 build_parse_very_complex_packet
        uint8_t packet[300] = {0};
        const uint8_t ones[8] = {1, 1, 1, 1, 1, 1, 1, 1}, twos[8] = {2, 2, 2, 2, 2, 2, 2, 2};
        const uint8_t pay[10] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10};
        const std::array<uint8_t, 16> z{};
        auto b = PacketBuilder<>(packet, 300).ethernet_qinq(M1, M2, 34525, 200, 100)
                     .ipv6(6, 5, 4, 3, 0, 255, z, z)
                     .hop_by_hop(60, 1, zp::Bytes{ones, 8})
                     .destination_options1(43, 1, zp::Bytes{ones, 8})
                     .routing_header(44, 1, 2, 3, zp::Bytes{twos, 8})
                     .fragment_header(51, 255, true, 0x04050607)
                     .authentication_header(60, 2, 305419896, 2271560481u, zp::Bytes{ones, 8})
                     .destination_options2(4, 1, zp::Bytes{ones, 8})
                     .ipv4(4, 5, 0, 0, 150, 0, 0, 0, 64, 6, IP1, IP2)
                     .tcp(IP1, 99, IP2, 11, 123, 321, 11, 99, 99, 4321, 1234, zp::Bytes{pay, 10});
        b.build(gpu.get());
        zp::PacketParser p = gpu.parse(zp::Bytes{packet, 300});
        CHECK(p.ethernet && p.ipv6 && p.ip_in_ip && p.tcp && !p.udp && !p.icmpv4 && !p.icmpv6);
        CHECK(p.ipv6->extension_headers.has_value());
        const auto& eh = *p.ipv6->extension_headers;
        CHECK(eh.hop_by_hop && eh.destination_1st && eh.routing && eh.fragment &&
              eh.auth_header && eh.destination_2nd);
        CHECK(p.ip_in_ip->kind == zp::IpInIp::Kind::Ipv4);
        CHECK(b.header_len() == 170 + 44);
        hex("build_parse_very_complex_packet", packet, 300);
        std::printf("OK build_parse_very_complex_packet\n");
    }
    {   // a step's Err: the reference's message (tcp.rs:109-111)
        uint8_t packet[64] = {0};
        const uint8_t big[30] = {0};
        bool thrown = false;
        try {
            PacketBuilder<>(packet, 64).ethernet(M1, M2, 2048)
                .ipv4(4, 5, 0, 0, 50, 0, 0, 0, 64, 6, IP1, IP2)
                .tcp(IP1, 1, IP2, 2, 3, 4, 5, 0, 2, 9, 0, zp::Bytes{big, 30}).build(gpu.get());
        } catch (const zp::BuildError& e) {
            thrown = e.code() == ZP_BERR_TCP_PAYLOAD &&
                     std::string(e.what()) == "Payload is too large to fit in the TCP packet.";
            CHECK(e.header_len() == 34);
        }
        CHECK(thrown);
        CHECK(packet[12] == 0x08 && packet[23] == 6);   // the Ok steps' bytes stay
        std::printf("OK build_error\n");
    }
    {   // zp::Ring: frames through the ring == the synchronous host batch
        std::vector<uint8_t> arena;
        std::vector<uint64_t> offs;
        std::vector<uint32_t> lens;
        for (int k = 0; k < 500; ++k) {
            uint8_t f[128] = {0};
            const uint16_t n = (uint16_t)(64 + (k * 7) % 60);
            PacketBuilder<>(f, n).ethernet(M1, M2, 2048)
                .ipv4(4, 5, 0, 0, (uint16_t)(n - 14), (uint16_t)k, 0, 0, 64, 17, IP1, IP2)
                .udp(IP1, (uint16_t)k, IP2, 53, (uint16_t)(n - 34)).build(gpu.get());
            offs.push_back(arena.size());
            lens.push_back(n);
            arena.insert(arena.end(), f, f + n);
        }
        std::vector<zp_record> want(offs.size());
        gpu.parse_batch(arena.data(), arena.size(), offs.data(), lens.data(), offs.size(), want.data());
        zp::Ring ring(0, 2, 8192, 64);
        size_t i = 0, done = 0, inflight = 0;
        while (done < offs.size()) {
            if (i < offs.size() && inflight < 2) {
                auto s = ring.acquire(10000);
                CHECK(s.has_value());
                size_t m = 0, pos = 0;
                while (i + m < offs.size() && m < 64 && pos + lens[i + m] <= 8192) {
                    std::memcpy(s->arena + pos, arena.data() + offs[i + m], lens[i + m]);
                    s->offs[m] = pos;
                    s->lens[m] = lens[i + m];
                    pos += lens[i + m];
                    ++m;
                }
                ring.submit(*s, m);
                i += m;
                ++inflight;
                continue;
            }
            auto d = ring.wait(10000);
            CHECK(d.has_value());
            CHECK(std::memcmp(d->records, want.data() + done, d->n * sizeof(zp_record)) == 0);
            done += d->n;
            --inflight;
            ring.release(*d);
        }
        for (const auto& r : want) CHECK(zp_rec_err(r) == 0 && (r.flags & ZP_F_UDP));
        std::printf("OK ring\n");
    }
    std::printf("ALL OK\n");
    return 0;
}
