// shapes.cpp — libnffshapes: the reference's two call shapes driven from many
// threads against a service of libnffacl, for bench.py's `call_shapes` record
// (bench code, not product: it measures the C-ABI from the outside).
//
//   scalar (burst == 0): T threads, each calling nffacl_service_classify one
//     packet at a time — pkt.L3ACLPort(rules) inside a SetSeparator function
//     (examples/firewall/firewall.go:54-57, examples/tutorial/step08.go:33-35);
//   burst (burst > 0): T threads (flow-function clones), each calling
//     nffacl_service_classify_burst with `burst` packets and waiting for the
//     answers — the VectorSeparateFunction shape of segmentProcess
//     (flow/flow.go:131, 1487-1520).
// Every verdict is compared with `expect` (the caller's oracle verdicts).
// The C-ABI entry points come in as function pointers taken from the library
// the caller loaded (so an experiment build under NFFACL_LIB is the one
// measured, never a second copy of libnffacl).
// Threads are pinned to NUMA node `pin_node` (>= 0) — nff-go pins every
// flow-function clone to a core (low.go:654-666), INTEGRATION.md puts them
// on the GPU's node.
#include <pthread.h>
#include <sched.h>
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "nffacl.h"

using Clock = std::chrono::steady_clock;

namespace {

bool node_cpus(int node, cpu_set_t &want) {
    CPU_ZERO(&want);
    cpu_set_t allowed;
    if (sched_getaffinity(0, sizeof allowed, &allowed) != 0) return false;
    std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
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
    return CPU_COUNT(&want) > 0;
}

double cpu_seconds() {
    rusage ru{};
    getrusage(RUSAGE_SELF, &ru);
    return ru.ru_utime.tv_sec + ru.ru_stime.tv_sec + 1e-6 * (ru.ru_utime.tv_usec + ru.ru_stime.tv_usec);
}

}  // namespace

extern "C" {

// out[0] Mpps, [1] p50 latency µs (per call), [2] p99 µs, [3] wrong verdicts,
// [4] calls, [5] process CPU µs per packet, [6] CPUs busy, [7] 1 if pinned,
// [8] calls that returned a status other than OK.
typedef int (*classify_fn)(nffacl_service *, const nffacl_rules *, const uint8_t *, uint32_t, uint32_t, uint32_t *);
typedef int (*burst_fn)(nffacl_service *, const nffacl_rules *, const uint8_t *const *, const uint32_t *, uint32_t,
                        uint32_t, uint32_t *);

__attribute__((visibility("default"))) int nffshapes_run(void *classify_p, void *burst_p, nffacl_service *svc,
                                                         const nffacl_rules *rules, const uint8_t *slots,
                                                         uint32_t stride, uint64_t n, const uint32_t *expect,
                                                         uint32_t threads, uint32_t burst, double seconds,
                                                         int pin_node, double *out) {
    const classify_fn nffacl_service_classify = reinterpret_cast<classify_fn>(classify_p);
    const burst_fn nffacl_service_classify_burst = reinterpret_cast<burst_fn>(burst_p);
    if (!classify_p || !burst_p || !svc || !rules || !slots || !expect || !out || n < 64 || threads == 0 || burst > 32)
        return -100;
    cpu_set_t want;
    const bool pin = pin_node >= 0 && node_cpus(pin_node, want);
    const uint32_t per = burst ? burst : 1;
    std::atomic<bool> go{false}, halt{false};
    std::atomic<uint64_t> total{0}, bad{0}, calls{0}, errs{0};
    std::atomic<uint32_t> ready{0};
    std::vector<std::vector<float>> lat(threads);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            if (pin) (void)pthread_setaffinity_np(pthread_self(), sizeof want, &want);
            std::vector<const uint8_t *> ptrs(per);
            std::vector<uint32_t> lens(per, stride), ports(per);
            uint64_t pos = (uint64_t(t) * 7919u * per) % (n - per);
            uint64_t done = 0, wrong = 0, c = 0, e = 0;
            lat[t].reserve(1 << 20);
            // first call outside the timing: mailbox assignment, table upload
            uint32_t p0 = 0;
            if (burst) {
                ptrs[0] = slots;
                (void)nffacl_service_classify_burst(svc, rules, ptrs.data(), lens.data(), 1, 0, &p0);
            } else {
                (void)nffacl_service_classify(svc, rules, slots, stride, 0, &p0);
            }
            ready.fetch_add(1);
            while (!go.load()) std::this_thread::yield();
            while (!halt.load(std::memory_order_relaxed)) {
                if (pos + per > n) pos = 0;
                int st;
                const auto t0 = Clock::now();
                if (burst) {
                    for (uint32_t i = 0; i < per; ++i) ptrs[i] = slots + (pos + i) * stride;
                    st = nffacl_service_classify_burst(svc, rules, ptrs.data(), lens.data(), per, 0, ports.data());
                } else {
                    st = nffacl_service_classify(svc, rules, slots + pos * stride, stride, 0, ports.data());
                }
                const auto t1 = Clock::now();
                if (lat[t].size() < (1u << 22)) lat[t].push_back(std::chrono::duration<float, std::micro>(t1 - t0).count());
                e += st != NFFACL_OK;
                for (uint32_t i = 0; i < per; ++i) wrong += ports[i] != expect[pos + i];
                done += per;
                ++c;
                pos += uint64_t(threads) * per;
                if (pos >= n) pos %= n;
            }
            total += done;
            bad += wrong;
            calls += c;
            errs += e;
        });
    while (ready.load() < threads) std::this_thread::yield();
    const double c0 = cpu_seconds();
    const auto t0 = Clock::now();
    go = true;
    std::this_thread::sleep_for(std::chrono::duration<double>(seconds));
    halt = true;
    for (auto &x : th) x.join();
    const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
    const double cpu = cpu_seconds() - c0;
    std::vector<float> all;
    for (auto &v : lat) all.insert(all.end(), v.begin(), v.end());
    std::sort(all.begin(), all.end());
    auto pct = [&](double p) { return all.empty() ? 0.0 : double(all[std::min(all.size() - 1, size_t(p * all.size()))]); };
    out[0] = double(total.load()) / dt / 1e6;
    out[1] = pct(0.5);
    out[2] = pct(0.99);
    out[3] = double(bad.load());
    out[4] = double(calls.load());
    out[5] = total.load() ? cpu / double(total.load()) * 1e6 : 0.0;
    out[6] = cpu / dt;
    out[7] = pin ? 1.0 : 0.0;
    out[8] = double(errs.load());
    return 0;
}

}  // extern "C"
