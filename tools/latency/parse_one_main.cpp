// Per-frame latency of zp_parse_one (PacketParser::parse for one frame,
// parser.rs:53, through the GPU: H2D -> kernel -> D2H -> sync), the drop-in
// for a caller that parses frame by frame. stdin: frame hex lines.
//   parse_one_main <threads> <calls per thread> [idle_us] [life_us]
// idle_us: zp_parse_one's mode (zp_parse_one_config): > 0 the resident server
// wave with that idle timeout (default 5000), 0 one kernel launch per call.
// Each thread owns one zp::Context (a zp_ctx may not be shared) and parses
// the frames round robin; prints mean / p50 / p99 microseconds per call and
// the aggregate calls per second.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

#include "zero_packet.hpp"

// diagnostic builds (-DZP_ONE_STAMPS) export the server's in-kernel stamps
extern "C" void zp__one_stamps(zp_ctx*, uint64_t*) __attribute__((weak));
// test hooks of libzp_hip.so: the server's life, its counters
extern "C" int zp__one_test_hooks(zp_ctx*, uint32_t, uint64_t, uint32_t) __attribute__((weak));
extern "C" int zp__one_stats(const zp_ctx*, uint64_t*) __attribute__((weak));

int main(int argc, char** argv) {
    const int threads = argc > 1 ? std::atoi(argv[1]) : 1;
    const int calls = argc > 2 ? std::atoi(argv[2]) : 2000;
    const uint32_t idle_us = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 5000u;
    const uint32_t life_us = argc > 4 ? (uint32_t)std::atoi(argv[4]) : 0u;   // 0: the default
    std::vector<uint64_t> stats(3 * threads, 0);
    std::vector<std::vector<uint8_t>> frames;
    std::string line;
    while (std::getline(std::cin, line)) {
        std::vector<uint8_t> v(line.size() / 2);
        for (size_t i = 0; i < v.size(); ++i) v[i] = (uint8_t)std::stoul(line.substr(2 * i, 2), nullptr, 16);
        frames.push_back(v);
    }
    std::vector<std::vector<double>> lat(threads);
    std::vector<int> bad(threads, 0);
    std::vector<double> busy(threads, 0);
    // every thread's timed loop starts together (after its context and
    // warm-up) and the rate is the calls over the span from the common
    // start to the last thread's end
    std::atomic<int> ready{0};
    std::vector<std::chrono::steady_clock::time_point> t_end(threads);
    std::chrono::steady_clock::time_point t_start;
    std::vector<std::vector<double>> st(5), ph(8);    // thread 0: bell->tile, tile->stores done, polls
    auto worker = [&](int t) {
        zp::Context ctx(0);
        ctx.parse_one_mode(idle_us);
        if (life_us && zp__one_test_hooks) zp__one_test_hooks(ctx.get(), life_us, 0, 0);
        for (int w = 0; w < 50; ++w) ctx.parse(zp::Bytes{frames[0].data(), frames[0].size()});
        lat[t].reserve(calls);
        if (ready.fetch_add(1) + 1 == threads) t_start = std::chrono::steady_clock::now();
        while (ready.load() < threads) {}
        const auto tb = std::chrono::steady_clock::now();
        for (int k = 0; k < calls; ++k) {
            const auto& f = frames[(k + t) % frames.size()];
            const auto t0 = std::chrono::steady_clock::now();
            zp::PacketParser p = ctx.parse(zp::Bytes{f.data(), f.size()});
            const auto t1 = std::chrono::steady_clock::now();
            if (!p.ethernet) ++bad[t];
            if (t == 0 && zp__one_stamps && idle_us) {
                uint64_t s4[14] = {0};
                zp__one_stamps(ctx.get(), s4);
                st[0].push_back((s4[1] - s4[0]) / 100.0);
                st[1].push_back((s4[2] - s4[1]) / 100.0);
                st[2].push_back((double)s4[3]);
                st[3].push_back((double)s4[4] / ((s4[1] - s4[0]) / 100.0));   // cycles per us
                st[4].push_back(s4[5] / 100.0);          // ZP_ONE_TWICE builds: the warm second pass
                for (int k = 1; k < 8; ++k)            // phase k end - bell (us)
                    ph[k].push_back(s4[6 + k] ? ((double)s4[6 + k] - (double)s4[0]) / 100.0 : -1.0);
            }
            lat[t].push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        t_end[t] = std::chrono::steady_clock::now();
        busy[t] = std::chrono::duration<double>(t_end[t] - tb).count();
        if (zp__one_stats) zp__one_stats(ctx.get(), &stats[3 * t]);
    };
    std::vector<std::thread> th;
    for (int t = 0; t < threads; ++t) th.emplace_back(worker, t);
    for (auto& x : th) x.join();
    // the concurrent span of the timed loops (context creation and warm-up
    // excluded): common start to the last thread's end
    double wall = 0;
    for (int t = 0; t < threads; ++t) {
        const double w = std::chrono::duration<double>(t_end[t] - t_start).count();
        wall = w > wall ? w : wall;
    }
    std::vector<double> all;
    for (auto& v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    double sum = 0;
    for (double x : all) sum += x;
    int nbad = 0;
    for (int b : bad) nbad += b;
    uint64_t tot[3] = {0, 0, 0};
    for (int t = 0; t < threads; ++t)
        for (int k = 0; k < 3; ++k) tot[k] += stats[3 * t + k];
    std::printf("{\"idle_us\": %u, \"life_us\": %u, \"threads\": %d, \"calls\": %zu, \"mean_us\": %.2f, "
                "\"p50_us\": %.2f, \"p99_us\": %.2f, \"calls_per_s\": %.0f, \"rejected\": %d, "
                "\"max_us\": %.1f, \"server_launches_rotations_relaunches\": [%llu, %llu, %llu]}\n",
                idle_us, life_us, threads, all.size(), sum / all.size(), all[all.size() / 2],
                all[(size_t)(all.size() * 0.99)], all.size() / wall, nbad, all.back(),
                (unsigned long long)tot[0], (unsigned long long)tot[1], (unsigned long long)tot[2]);
    if (!st[0].empty()) {
        for (auto& v : st) std::sort(v.begin(), v.end());
        std::printf("{\"server_stamps_p50\": {\"bell_to_tile_us\": %.2f, \"tile_to_stores_done_us\": %.2f, "
                    "\"polls\": %.0f, \"shader_mhz\": %.0f, \"second_pass_us\": %.2f}}\n",
                    st[0][st[0].size() / 2], st[1][st[1].size() / 2], st[2][st[2].size() / 2],
                    st[3][st[3].size() / 2], st[4][st[4].size() / 2]);
        std::printf("{\"server_phase_end_after_bell_us_p50\": [");
        for (int k = 1; k < 8; ++k) {
            std::sort(ph[k].begin(), ph[k].end());
            std::printf("%s%.2f", k > 1 ? ", " : "", ph[k][ph[k].size() / 2]);
        }
        std::printf("], \"phases\": \"1 setup, 2 first issue, 3 stream done, 4 tile done, 5 walk, 6 verdict, 7 -\"}\n");
    }
    return nbad ? 1 : 0;
}
