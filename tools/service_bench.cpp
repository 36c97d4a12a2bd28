// service_bench — the reference's scalar call shape through the C++ mirror:
// T threads (flow-function clones) each calling flow::ACLSplitter(rules) —
// pkt.L3ACLPort(rules), one packet per call (examples/tutorial/step08.go:33-35,
// examples/firewall/firewall.go:54-57) — answered by the GPU's persistent
// consumer (nffacl_service_*).  Every answer is checked against the oracle's
// verdict for that packet (expect.bin, written by tools/service_bench.py).
//
//   service_bench RULES SLOTS EXPECT THREADS SECONDS
// prints one JSON line.
#include <sched.h>
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "nffgo.hpp"

using namespace nffgo;
using Clock = std::chrono::steady_clock;

static std::vector<uint8_t> slurp(const char *path) {
    std::ifstream f(path, std::ios::binary);
    return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

int main(int argc, char **argv) {
    if (argc != 6) {
        std::fprintf(stderr, "usage: %s RULES SLOTS EXPECT THREADS SECONDS\n", argv[0]);
        return 2;
    }
    const uint32_t stride = 80, threads = std::atoi(argv[4]);
    const double seconds = std::atof(argv[5]);
    const std::vector<uint8_t> slots = slurp(argv[2]), ex = slurp(argv[3]);
    const size_t n = slots.size() / stride;
    if (ex.size() != n * 4) {
        std::fprintf(stderr, "expect.bin: %zu bytes for %zu packets\n", ex.size(), n);
        return 1;
    }
    const uint32_t *expect = reinterpret_cast<const uint32_t *>(ex.data());
    auto loaded = packet::GetL3ACLFromTextTable(argv[1]);
    if (loaded.second) {
        std::fprintf(stderr, "rules: %s\n", loaded.second->Error().c_str());
        return 1;
    }
    std::shared_ptr<const packet::L3Rules> rules = loaded.first;
    rules->Prepare();
    std::vector<packet::Packet> pk(n);
    for (size_t i = 0; i < n; ++i) pk[i] = packet::Packet{slots.data() + i * stride, stride};
    // NFFACL_BENCH_PIN=1: run every caller on the GPU's NUMA node (the
    // deployment INTEGRATION.md recommends: flow-function lcores pinned there)
    const int gpu_node = nffacl_device_numa_node(packet::ACLDevice());
    bool pinned = false;
    if (const char *pin = std::getenv("NFFACL_BENCH_PIN"); pin && std::atoi(pin) == 1 && gpu_node >= 0) {
        cpu_set_t allowed, want;
        CPU_ZERO(&want);
        if (sched_getaffinity(0, sizeof allowed, &allowed) == 0) {
            std::ifstream f("/sys/devices/system/node/node" + std::to_string(gpu_node) + "/cpulist");
            std::string list;
            std::getline(f, list);
            size_t i = 0;
            while (i < list.size()) {  // "a-b,c,d-e"
                size_t j = list.find(',', i);
                if (j == std::string::npos) j = list.size();
                const std::string r = list.substr(i, j - i);
                const size_t dash = r.find('-');
                const int a = std::atoi(r.c_str()), b = dash == std::string::npos ? a : std::atoi(r.c_str() + dash + 1);
                for (int c = a; c <= b && c < CPU_SETSIZE; ++c)
                    if (CPU_ISSET(c, &allowed)) CPU_SET(c, &want);
                i = j + 1;
            }
            pinned = CPU_COUNT(&want) > 0 && sched_setaffinity(0, sizeof want, &want) == 0;
        }
    }
    const flow::SplitFunction split = flow::ACLSplitter(rules);
    (void)split(&pk[0]);  // first call: consumer launch + table descriptor

    std::atomic<bool> go{false}, halt{false};
    std::atomic<uint64_t> total{0}, bad{0};
    std::vector<std::vector<float>> lat(threads);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            size_t pos = (size_t(t) * 7919) % n;
            uint64_t done = 0, wrong = 0;
            lat[t].reserve(1 << 20);
            while (!go.load()) std::this_thread::yield();
            while (!halt.load(std::memory_order_relaxed)) {
                const auto t0 = Clock::now();
                const uint32_t port = split(&pk[pos]);
                const auto t1 = Clock::now();
                if (lat[t].size() < (1u << 22)) lat[t].push_back(std::chrono::duration<float, std::micro>(t1 - t0).count());
                wrong += port != expect[pos];
                ++done;
                pos += threads;
                if (pos >= n) pos -= n;
            }
            total += done;
            bad += wrong;
        });
    auto cpu_s = [] {
        rusage ru{};
        getrusage(RUSAGE_SELF, &ru);
        return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
    };
    const double c0 = cpu_s();
    const auto t0 = Clock::now();
    go = true;
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    halt = true;
    for (auto &x : th) x.join();
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    const double cpu = cpu_s() - c0;  // process CPU seconds over the run (all threads)
    std::string quota = "?";  // cgroup v2 CPU bandwidth limit ("max" or "QUOTA PERIOD")
    {
        std::ifstream q("/sys/fs/cgroup/cpu.max");
        if (q) std::getline(q, quota);
    }
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : double(all[std::min(all.size() - 1, size_t(p * all.size()))]); };
    nffacl_service_stats st{};
    nffacl_service_get_stats(packet::detail::service(packet::ACLDevice()), &st);
    std::printf("{\"threads\": %u, \"calls\": %llu, \"mpps\": %.3f, \"lat_us_p50\": %.2f, \"lat_us_p90\": %.2f, "
                "\"lat_us_p99\": %.2f, \"lat_us_p999\": %.1f, \"wrong\": %llu, \"launches\": %llu, "
                "\"timeouts\": %llu, \"polls\": %llu, \"poll_ns\": %.0f, \"groups\": %llu, \"group_ns\": %.0f, "
                "\"answered\": %llu, \"cpu_us_per_call\": %.2f, \"cpus_busy\": %.2f, \"cpu_max\": \"%s\", "
                "\"gpu_node\": %d, \"pinned\": %s}\n",
                threads, (unsigned long long)total.load(), total.load() / dt / 1e6, pct(0.5), pct(0.9), pct(0.99),
                pct(0.999), (unsigned long long)bad.load(), (unsigned long long)st.launches,
                (unsigned long long)st.timeouts, (unsigned long long)st.polls, st.poll_ns,
                (unsigned long long)st.groups, st.group_ns, (unsigned long long)st.answered,
                total.load() ? cpu / double(total.load()) * 1e6 : 0.0, cpu / dt, quota.c_str(), gpu_node,
                pinned ? "true" : "false");
    return bad.load() ? 1 : 0;
}
