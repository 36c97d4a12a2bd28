// batcher_bench — host-ingest throughput/latency of nffacl_batcher.
//
// T producer threads play the reference's flow-function clones: each loops
// over bursts of B packets (the 32-packet bursts of segmentProcess,
// flow/flow.go:1487-1520), calls nffacl_batcher_classify (submit + wait) and
// records the burst's latency.  Packets are pointers into a host buffer of
// pre-built frames (rules text + raw slots written by tools/batcher_bench.py).
//
//   batcher_bench RULES SLOTS STRIDE THREADS BURST MAX_BATCH DELAY_US SECONDS
// prints one JSON line.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "nffacl.h"

using Clock = std::chrono::steady_clock;

int main(int argc, char **argv) {
    if (argc != 9) {
        std::fprintf(stderr, "usage: %s RULES SLOTS STRIDE THREADS BURST MAX_BATCH DELAY_US SECONDS\n", argv[0]);
        return 2;
    }
    const uint32_t stride = std::atoi(argv[3]), threads = std::atoi(argv[4]), burst = std::atoi(argv[5]);
    const uint32_t max_batch = std::atoi(argv[6]), delay = std::atoi(argv[7]);
    const double seconds = std::atof(argv[8]);
    std::ifstream f(argv[2], std::ios::binary);
    std::vector<uint8_t> slots((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const size_t n = slots.size() / stride;
    nffacl_rules *rules = nullptr;
    char err[256];
    if (nffacl_rules_load_text(argv[1], &rules, err, sizeof err) != NFFACL_OK) {
        std::fprintf(stderr, "rules: %s\n", err);
        return 1;
    }
    nffacl_engine *eng = nullptr;
    if (nffacl_engine_create(0, rules, &eng) != NFFACL_OK) {
        std::fprintf(stderr, "engine: %s\n", nffacl_last_error());
        return 1;
    }
    nffacl_batcher *b = nullptr;
    if (nffacl_batcher_create(eng, stride, max_batch, delay, 4, &b) != NFFACL_OK) {
        std::fprintf(stderr, "batcher: %s\n", nffacl_last_error());
        return 1;
    }
    std::vector<const uint8_t *> ptrs(n);
    std::vector<uint32_t> lens(n, stride);
    for (size_t i = 0; i < n; ++i) ptrs[i] = slots.data() + i * stride;

    std::atomic<bool> go{false}, halt{false};
    std::atomic<uint64_t> total{0};
    std::atomic<int> failed{0};
    std::vector<std::vector<float>> lat(threads);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            std::vector<uint32_t> ports(burst);
            size_t pos = (size_t(t) * 7919 * burst) % (n - burst);
            uint64_t done = 0;
            while (!go.load()) std::this_thread::yield();
            while (!halt.load(std::memory_order_relaxed)) {
                const auto t0 = Clock::now();
                if (nffacl_batcher_classify(b, &ptrs[pos], &lens[pos], burst, ports.data()) != NFFACL_OK) {
                    failed = 1;
                    break;
                }
                lat[t].push_back(std::chrono::duration<float, std::micro>(Clock::now() - t0).count());
                done += burst;
                pos += size_t(threads) * burst;
                if (pos + burst > n) pos = (pos + burst) % (n - burst);
            }
            total += done;
        });
    const auto t0 = Clock::now();
    go = true;
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    halt = true;
    for (auto &x : th) x.join();
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : double(all[std::min(all.size() - 1, size_t(p * all.size()))]); };
    nffacl_batcher_stats st{};
    nffacl_batcher_get_stats(b, &st);
    std::printf("{\"threads\": %u, \"burst\": %u, \"max_batch\": %u, \"delay_us\": %u, \"stride\": %u, "
                "\"mpps\": %.2f, \"lat_us_p50\": %.1f, \"lat_us_p99\": %.1f, \"batches\": %llu, "
                "\"mean_batch\": %.1f, \"timeouts\": %llu, \"failed\": %d}\n",
                threads, burst, max_batch, delay, stride, total.load() / dt / 1e6, pct(0.5), pct(0.99),
                (unsigned long long)st.batches, st.batches ? double(st.packets) / st.batches : 0.0,
                (unsigned long long)st.timeouts, failed.load());
    nffacl_batcher_destroy(b);
    nffacl_engine_destroy(eng);
    nffacl_rules_free(rules);
    return failed.load();
}
