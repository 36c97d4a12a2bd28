// nffgo.hpp — C++ host mirror of the nff-go API surface this path replaces,
// layered on the libnffacl C-ABI (include/nffacl.h).  Header-only.
//
// The reference host code is Go; with no Go toolchain in this image the host
// side above the C-ABI is C++ and mirrors the reference's names, argument
// meaning and error behaviour, so code written against nff-go reads the same:
//
//   nffgo::common::NFError / ErrorCode          common/error.go:18-66
//   nffgo::packet::GetL3ACLFromTextTable         packet/acl.go:148-178
//   nffgo::packet::GetL3ACLFromJSON              packet/acl.go:121-134
//   nffgo::packet::L3Rules                       packet/acl.go:451-455
//   nffgo::packet::Packet::L3ACLPermit / Port    packet/acl.go:495-506
//   nffgo::flow::SeparateFunction / SplitFunction flow/flow.go:128, 134
//   nffgo::flow::ACLSeparator / ACLSplitter      the scalar separator of
//                                                examples/firewall/firewall.go:54-57
//   nffgo::flow::RulesPointer                    the atomic *L3Rules of
//                                                examples/tutorial/step08.go:9, 33-44
//   nffgo::flow::VectorSeparateFunction          flow/flow.go:131
//   nffgo::flow::ACLVectorSeparator              the vector separator body of
//                                                testSingleWorkingFF.go:538-546
//   nffgo::flow::Aggregator                      burst aggregation for GPU-size batches
//
// Every verdict is computed by the HIP kernels of libnffacl; there is no CPU
// path.  Packet::L3ACLPort / L3ACLPermit — one packet per call, the rule set
// passed per call, as in the reference — go through the per-GPU persistent
// consumer (nffacl_service_*: one PCIe round trip, no kernel launch), against
// the table the rule set itself owns (nffacl_rules_prepare), so a rule reload
// is the reference's "load new rules, swap the pointer" and nothing else.
// Bursts go through a shared batcher (ACLVectorSeparator) or an Aggregator.
// The GPU is the one nearest the calling thread (nffacl_local_device), or the
// one SetACLDevice chose.
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "nffacl.h"

namespace nffgo {

namespace common {

// common/error.go:18-50 (values identical).
enum class ErrorCode : int {
    Fail = 1,
    ParseRuleJSONErr = 11,
    FileErr = 12,
    ParseRuleErr = 13,
    IncorrectArgInRules = 14,
    IncorrectRule = 15,
};

// common/error.go:54-66: Error() formats "<message> (<code>)".
struct NFError {
    ErrorCode Code = ErrorCode::Fail;
    std::string Message;
    std::string Error() const { return Message; }
};

inline NFError from_status(int st, const std::string &msg) {
    NFError e;
    e.Code = (st <= -11 && st >= -15) ? static_cast<ErrorCode>(-st) : ErrorCode::Fail;
    e.Message = msg;
    return e;
}

}  // namespace common

namespace types {
// types/const.go:22-45, 66-78 — the constants the ACL path depends on.
constexpr uint16_t IPV4Number = 0x0800, IPV6Number = 0x86dd, ARPNumber = 0x0806;
constexpr uint8_t ICMPNumber = 0x01, TCPNumber = 0x06, UDPNumber = 0x11, ICMPv6Number = 0x3a;
constexpr uint32_t EtherLen = 14, IPv4MinLen = 20, IPv6Len = 40, TCPMinLen = 20, UDPLen = 8, ICMPLen = 8;
using IPv4Address = uint32_t;                  // types/ipv4.go:13 (LE of wire bytes)
using IPv6Address = std::array<uint8_t, 16>;   // types/ipv6.go:13
}  // namespace types

namespace packet {

// GPU the mirror's calls use: -1 = the one nearest the calling thread
// (nffacl_local_device), else the device set here (once, at start-up, as a
// Go program would pass it to flow.SystemInit).
inline std::atomic<int> &acl_device_setting() {
    static std::atomic<int> dev{-1};
    return dev;
}
inline void SetACLDevice(int dev) { acl_device_setting().store(dev); }
inline int ACLDevice() {
    const int d = acl_device_setting().load(std::memory_order_relaxed);
    return d >= 0 ? d : nffacl_local_device();
}

// Owner of an nffacl_rules handle plus, lazily, its compiled device table.
class L3Rules {
public:
    explicit L3Rules(nffacl_rules *h) : h_(h) {}
    L3Rules(const L3Rules &) = delete;
    L3Rules &operator=(const L3Rules &) = delete;
    ~L3Rules() {
        if (eng_) nffacl_engine_destroy(eng_);
        if (h_) nffacl_rules_free(h_);
    }
    const nffacl_rules *handle() const { return h_; }

    // The reference's unexported ip4/ip6 slices, as the records libnffacl holds.
    std::vector<nffacl_rule4> ip4() const {
        size_t n4 = 0, n6 = 0;
        nffacl_rules_counts(h_, &n4, &n6);
        std::vector<nffacl_rule4> v(n4);
        for (size_t i = 0; i < n4; ++i) nffacl_rules_get4(h_, i, &v[i]);
        return v;
    }
    std::vector<nffacl_rule6> ip6() const {
        size_t n4 = 0, n6 = 0;
        nffacl_rules_counts(h_, &n4, &n6);
        std::vector<nffacl_rule6> v(n6);
        for (size_t i = 0; i < n6; ++i) nffacl_rules_get6(h_, i, &v[i]);
        return v;
    }

    // Compile + upload the rule set's own table on the ACL device now (the
    // first per-packet call does it otherwise): call it where the rules are
    // loaded, as step08's reload goroutine would.
    void Prepare() const {
        const int st = nffacl_rules_prepare(h_, ACLDevice());
        if (st != NFFACL_OK)
            throw std::runtime_error(std::string("nffacl_rules_prepare: ") + nffacl_strerror(st) + " " +
                                     nffacl_last_error());
    }

    // Engine (bulk host pipeline) on the ACL device (first use compiles + uploads).
    nffacl_engine *engine(int algo = NFFACL_ALGO_AUTO) const {
        std::call_once(once_, [&] {
            st_ = nffacl_engine_create_ex(ACLDevice(), h_, algo, &eng_);
            if (st_ != NFFACL_OK) err_ = nffacl_last_error();
        });
        if (st_ != NFFACL_OK)
            throw std::runtime_error(std::string("nffacl_engine_create: ") + nffacl_strerror(st_) + " " + err_);
        return eng_;
    }

    // L3Rules{ip4: ..., ip6: ...} literal, as the reference tests build them.
    static std::shared_ptr<L3Rules> FromRecords(const std::vector<nffacl_rule4> &ip4,
                                                const std::vector<nffacl_rule6> &ip6) {
        nffacl_rules *h = nullptr;
        const int st = nffacl_rules_from_arrays(ip4.data(), ip4.size(), ip6.data(), ip6.size(), &h);
        if (st != NFFACL_OK) throw std::runtime_error("nffacl_rules_from_arrays failed");
        return std::make_shared<L3Rules>(h);
    }

private:
    nffacl_rules *h_ = nullptr;
    mutable std::once_flag once_;
    mutable nffacl_engine *eng_ = nullptr;
    mutable int st_ = NFFACL_OK;
    mutable std::string err_;
};

using RulesOrError = std::pair<std::shared_ptr<L3Rules>, std::optional<common::NFError>>;

namespace detail {
template <class F>
RulesOrError load(F fn, const std::string &filename) {
    nffacl_rules *h = nullptr;
    char err[512] = {0};
    const int st = fn(filename.c_str(), &h, err, sizeof err);
    if (st != NFFACL_OK) return {nullptr, common::from_status(st, err)};
    return {std::make_shared<L3Rules>(h), std::nullopt};
}
}  // namespace detail

// acl.go:148.  On error the rules pointer is null (the reference also hands
// back a partly filled *L3Rules, acl.go:177, that no caller uses).
inline RulesOrError GetL3ACLFromTextTable(const std::string &filename) {
    return detail::load(nffacl_rules_load_text, filename);
}

// acl.go:121.
inline RulesOrError GetL3ACLFromJSON(const std::string &filename) {
    return detail::load(nffacl_rules_load_json, filename);
}

// Slot width handed to the GPU: the verdict reads wire bytes 12..77, so 80
// bytes keep IPv4 headers with IHL up to 15 exact.
constexpr uint32_t kSlot = 80;

// A packet as the ACL sees it: the frame bytes starting at the Ethernet
// header (packet.go:207-218 Ether pointer + data length).
struct Packet {
    const uint8_t *Ether = nullptr;
    uint32_t Len = 0;

    uint32_t L3ACLPort(const L3Rules &rules) const;   // acl.go:504
    bool L3ACLPermit(const L3Rules &rules) const {    // acl.go:495
        return L3ACLPort(rules) > 0;
    }
    uint32_t L2ACLPort(const class L2Rules &rules) const;  // acl.go:472
    bool L2ACLPermit(const class L2Rules &rules) const;    // acl.go:464
};

// Classify n packets in one GPU call (host staging inside libnffacl).
inline void L3ACLPortBatch(const Packet *const *pkts, size_t n, uint32_t *ports, const L3Rules &rules) {
    if (n == 0) return;
    std::vector<uint8_t> slots(n * kSlot, 0);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t len = pkts[i]->Len < kSlot ? pkts[i]->Len : kSlot;
        if (len) std::memcpy(&slots[i * kSlot], pkts[i]->Ether, len);
    }
    const int st = nffacl_classify_host(rules.engine(), slots.data(), kSlot, n, ports, nullptr);
    if (st != NFFACL_OK)
        throw std::runtime_error(std::string("nffacl_classify_host: ") + nffacl_strerror(st) + " " +
                                 nffacl_last_error());
}

namespace detail {
// One persistent consumer per GPU for the whole process (nffacl_service_*):
// scalar mailboxes (burst = false) or burst mailboxes (one per clone).
inline nffacl_service *service(int dev, bool burst = false) {
    struct Holder {
        std::once_flag once;
        nffacl_service *svc = nullptr;
        int st = NFFACL_OK;
        ~Holder() {
            if (svc) nffacl_service_destroy(svc);
        }
    };
    static Holder holders[2][16];
    if (dev < 0 || dev >= 16) throw std::runtime_error("ACL device out of range");
    Holder &h = holders[burst ? 1 : 0][dev];
    std::call_once(h.once, [&] {
        h.st = burst ? nffacl_service_create_burst(dev, 0, 2000, &h.svc) : nffacl_service_create(dev, 0, 2000, &h.svc);
    });
    if (h.st != NFFACL_OK)
        throw std::runtime_error(std::string("nffacl_service_create: ") + nffacl_strerror(h.st) + " " +
                                 nffacl_last_error());
    return h.svc;
}

// The service failure policy (nffacl.h): a call the consumer did not answer
// (twice) returns NFFACL_ERR_TIMEOUT with verdict 0 — reject, what l3ACL
// gives a packet no rule matches — and is counted in the service's stats.
// The reference's verdict path never errors (acl.go:522-565), so the mirror
// returns that verdict instead of throwing out of a flow function; any other
// status is a programming error and throws.
inline void check_service(int st, const char *what) {
    if (st != NFFACL_OK && st != NFFACL_ERR_TIMEOUT)
        throw std::runtime_error(std::string(what) + ": " + nffacl_strerror(st) + " " + nffacl_last_error());
}
}  // namespace detail

// acl.go:504 for one packet: the calling thread's mailbox of the GPU's
// persistent consumer, against the rule set's own table.
inline uint32_t Packet::L3ACLPort(const L3Rules &rules) const {
    uint32_t port = 0;
    detail::check_service(nffacl_service_classify(detail::service(ACLDevice()), rules.handle(), Ether, Len, 0, &port),
                          "nffacl_service_classify");
    return port;
}

// L3ACLPort of a burst (the VectorSeparateFunction shape, flow.go:131): one
// request per 32 packets to this thread's burst mailbox of the GPU's
// consumer — one PCIe round trip per burst, no kernel launch.
inline void L3ACLPortBurst(const Packet *const *pkts, size_t n, uint32_t *ports, const L3Rules &rules) {
    const uint8_t *frames[32];
    uint32_t lens[32];
    nffacl_service *svc = detail::service(ACLDevice(), true);
    for (size_t off = 0; off < n; off += 32) {
        const size_t m = std::min<size_t>(32, n - off);
        for (size_t i = 0; i < m; ++i) {
            frames[i] = pkts[off + i]->Ether;
            lens[i] = pkts[off + i]->Len;
        }
        detail::check_service(nffacl_service_classify_burst(svc, rules.handle(), frames, lens,
                                                            static_cast<uint32_t>(m), 0, ports + off),
                              "nffacl_service_classify_burst");
    }
}

// ---- L2 ACL (acl.go:68-117, 356-383, 457-491) ----------------------------------

// Owner of an nffacl_l2rules handle plus, lazily, its device table.
class L2Rules {
public:
    explicit L2Rules(nffacl_l2rules *h) : h_(h) {}
    L2Rules(const L2Rules &) = delete;
    L2Rules &operator=(const L2Rules &) = delete;
    ~L2Rules() {
        if (eng_) nffacl_l2_engine_destroy(eng_);
        if (h_) nffacl_l2rules_free(h_);
    }
    const nffacl_l2rules *handle() const { return h_; }

    // The reference's unexported eth slice (acl.go:458-460).
    std::vector<nffacl_l2_rule> eth() const {
        size_t n = 0;
        nffacl_l2rules_count(h_, &n);
        std::vector<nffacl_l2_rule> v(n);
        for (size_t i = 0; i < n; ++i) nffacl_l2rules_get(h_, i, &v[i]);
        return v;
    }

    nffacl_l2engine *engine() const {
        std::call_once(once_, [&] {
            st_ = nffacl_l2_engine_create(ACLDevice(), h_, &eng_);
            if (st_ != NFFACL_OK) err_ = nffacl_last_error();
        });
        if (st_ != NFFACL_OK)
            throw std::runtime_error(std::string("nffacl_l2_engine_create: ") + nffacl_strerror(st_) + " " + err_);
        return eng_;
    }

    // L2Rules{eth: ...} literal (acl_internal_test.go:1189-1191).
    static std::shared_ptr<L2Rules> FromRecords(const std::vector<nffacl_l2_rule> &eth) {
        nffacl_l2rules *h = nullptr;
        if (nffacl_l2rules_from_array(eth.data(), eth.size(), &h) != NFFACL_OK)
            throw std::runtime_error("nffacl_l2rules_from_array failed");
        return std::make_shared<L2Rules>(h);
    }

private:
    nffacl_l2rules *h_ = nullptr;
    mutable std::once_flag once_;
    mutable nffacl_l2engine *eng_ = nullptr;
    mutable int st_ = NFFACL_OK;
    mutable std::string err_;
};

using L2RulesOrError = std::pair<std::shared_ptr<L2Rules>, std::optional<common::NFError>>;

namespace detail {
template <class F>
L2RulesOrError load_l2(F fn, const std::string &filename) {
    nffacl_l2rules *h = nullptr;
    char err[512] = {0};
    const int st = fn(filename.c_str(), &h, err, sizeof err);
    if (st != NFFACL_OK) return {nullptr, common::from_status(st, err)};
    return {std::make_shared<L2Rules>(h), std::nullopt};
}
}  // namespace detail

// acl.go:88.
inline L2RulesOrError GetL2ACLFromTextTable(const std::string &filename) {
    return detail::load_l2(nffacl_l2rules_load_text, filename);
}

// acl.go:70.
inline L2RulesOrError GetL2ACLFromJSON(const std::string &filename) {
    return detail::load_l2(nffacl_l2rules_load_json, filename);
}

// L2ACLPort over n packets in one GPU call (only the Ethernet header travels).
inline void L2ACLPortBatch(const Packet *const *pkts, size_t n, uint32_t *ports, const L2Rules &rules) {
    if (n == 0) return;
    constexpr uint32_t kL2Slot = 64;
    std::vector<uint8_t> slots(n * kL2Slot, 0);
    for (size_t i = 0; i < n; ++i) {
        const uint32_t len = pkts[i]->Len < types::EtherLen ? pkts[i]->Len : types::EtherLen;
        if (len) std::memcpy(&slots[i * kL2Slot], pkts[i]->Ether, len);
    }
    const int st = nffacl_l2_classify_host(rules.engine(), slots.data(), kL2Slot, n, ports, nullptr);
    if (st != NFFACL_OK)
        throw std::runtime_error(std::string("nffacl_l2_classify_host: ") + nffacl_strerror(st) + " " +
                                 nffacl_last_error());
}

inline bool Packet::L2ACLPermit(const L2Rules &rules) const { return L2ACLPort(rules) > 0; }

inline uint32_t Packet::L2ACLPort(const L2Rules &rules) const {
    const Packet *p = this;
    uint32_t port = 0;
    L2ACLPortBatch(&p, 1, &port, rules);
    return port;
}

}  // namespace packet

namespace flow {

constexpr int vBurstSize = 32;  // flow/flow.go:465-469

// flow.go:128 / 134: the per-packet user functions SetSeparator / SetSplitter call.
using SeparateFunction = std::function<bool(packet::Packet *pkt)>;
using SplitFunction = std::function<uint32_t(packet::Packet *pkt)>;

// flow.go:131: VectorSeparateFunction(pkts, mask, answers, ctx)
using VectorSeparateFunction =
    std::function<void(packet::Packet *const *pkts, const bool *mask, bool *answers)>;
using VectorSplitFunction =  // flow.go:139
    std::function<void(packet::Packet *const *pkts, const bool *mask, uint8_t *answers)>;

// The reference's vector separator over L3ACLPermit
// (testSingleWorkingFF.go:538-546) as one request per burst to the GPU's
// resident consumer (packet::L3ACLPortBurst).
inline VectorSeparateFunction ACLVectorSeparator(std::shared_ptr<const packet::L3Rules> rules) {
    return [rules](packet::Packet *const *pkts, const bool *mask, bool *answers) {
        const packet::Packet *sel[vBurstSize];
        int idx[vBurstSize];
        size_t n = 0;
        for (int i = 0; i < vBurstSize; ++i)
            if (mask[i] && pkts[i]) { sel[n] = pkts[i]; idx[n++] = i; }
        uint32_t ports[vBurstSize] = {0};
        packet::L3ACLPortBurst(sel, n, ports, *rules);
        for (size_t k = 0; k < n; ++k) answers[idx[k]] = ports[k] > 0;
    };
}

// vectorL3Splitter (testSingleWorkingFF.go:553-560): answers[i] = uint8(L3ACLPort).
inline VectorSplitFunction ACLVectorSplitter(std::shared_ptr<const packet::L3Rules> rules) {
    return [rules](packet::Packet *const *pkts, const bool *mask, uint8_t *answers) {
        const packet::Packet *sel[vBurstSize];
        int idx[vBurstSize];
        size_t n = 0;
        for (int i = 0; i < vBurstSize; ++i)
            if (mask[i] && pkts[i]) { sel[n] = pkts[i]; idx[n++] = i; }
        uint32_t ports[vBurstSize] = {0};
        packet::L3ACLPortBurst(sel, n, ports, *rules);
        for (size_t k = 0; k < n; ++k) answers[idx[k]] = static_cast<uint8_t>(ports[k]);
    };
}

// One nffacl_batcher per GPU, shared by every flow-function clone: the
// clones' bursts ride in common GPU batches.
// The device form takes the rule set per burst (the reference's per-call
// *L3Rules); the engine form classifies against one engine's active table.
class SharedBatcher {
public:
    explicit SharedBatcher(int device = -1, uint32_t max_batch = 1 << 16, uint32_t max_delay_us = 100,
                           uint32_t nbuf = 4) {
        const int st = nffacl_batcher_create_device(device >= 0 ? device : packet::ACLDevice(), packet::kSlot,
                                                    max_batch, max_delay_us, nbuf, &b_);
        if (st != NFFACL_OK)
            throw std::runtime_error(std::string("nffacl_batcher_create_device: ") + nffacl_strerror(st));
    }
    SharedBatcher(std::shared_ptr<const packet::L3Rules> rules, uint32_t max_batch = 1 << 16,
                  uint32_t max_delay_us = 100, uint32_t nbuf = 4)
        : rules_(std::move(rules)) {
        const int st = nffacl_batcher_create(rules_->engine(), packet::kSlot, max_batch, max_delay_us, nbuf, &b_);
        if (st != NFFACL_OK)
            throw std::runtime_error(std::string("nffacl_batcher_create: ") + nffacl_strerror(st));
    }
    SharedBatcher(const SharedBatcher &) = delete;
    SharedBatcher &operator=(const SharedBatcher &) = delete;
    ~SharedBatcher() { nffacl_batcher_destroy(b_); }

    // L3ACLPort of n packets against `rules` (device form), or the engine's
    // table (rules == nullptr, engine form); blocks until their batch is back.
    void Classify(const packet::L3Rules *rules, const packet::Packet *const *pkts, size_t n, uint32_t *ports) {
        const uint8_t *frames[vBurstSize];
        uint32_t lens[vBurstSize];
        for (size_t off = 0; off < n; off += vBurstSize) {
            const size_t m = std::min<size_t>(vBurstSize, n - off);
            for (size_t i = 0; i < m; ++i) {
                frames[i] = pkts[off + i]->Ether;
                lens[i] = pkts[off + i]->Len;
            }
            const int st = rules ? nffacl_batcher_classify_rules(b_, rules->handle(), frames, lens,
                                                                 static_cast<uint32_t>(m), ports + off)
                                 : nffacl_batcher_classify(b_, frames, lens, static_cast<uint32_t>(m), ports + off);
            if (st != NFFACL_OK)
                throw std::runtime_error(std::string("nffacl_batcher_classify: ") + nffacl_strerror(st) + " " +
                                         nffacl_last_error());
        }
    }
    void Classify(const packet::Packet *const *pkts, size_t n, uint32_t *ports) { Classify(nullptr, pkts, n, ports); }
    nffacl_batcher_stats Stats() const {
        nffacl_batcher_stats s{};
        nffacl_batcher_get_stats(b_, &s);
        return s;
    }

private:
    std::shared_ptr<const packet::L3Rules> rules_;  // engine form: keeps the engine alive
    nffacl_batcher *b_ = nullptr;
};

// firewall.go:54-57's l3Separator for SetSeparator: pkt.L3ACLPermit(rules)
// per call, answered by the GPU's persistent consumer.
inline SeparateFunction ACLSeparator(std::shared_ptr<const packet::L3Rules> rules) {
    return [rules](packet::Packet *pkt) { return pkt->L3ACLPermit(*rules); };
}
// SetSplitter's per-packet L3ACLPort (examples/forwarding/forwarding.go:49-67).
inline SplitFunction ACLSplitter(std::shared_ptr<const packet::L3Rules> rules) {
    return [rules](packet::Packet *pkt) { return pkt->L3ACLPort(*rules); };
}

// step08.go's `rulesp unsafe.Pointer`: the rule set user code swaps while
// clones classify (atomic.StorePointer / LoadPointer, step08.go:33-44).  A
// clone loads the pointer once per call and classifies against exactly that
// rule set; the old one is freed when its last user drops it (Go's GC).
class RulesPointer {
public:
    explicit RulesPointer(std::shared_ptr<const packet::L3Rules> r) : p_(std::move(r)) {}
    std::shared_ptr<const packet::L3Rules> Load() const { return std::atomic_load(&p_); }
    void Store(std::shared_ptr<const packet::L3Rules> r) { std::atomic_store(&p_, std::move(r)); }

private:
    std::shared_ptr<const packet::L3Rules> p_;
};

// step08.go:33-35's mySplitter: L3ACLPort against the current rule set.
inline SplitFunction ACLSplitter(std::shared_ptr<RulesPointer> rulesp) {
    return [rulesp](packet::Packet *pkt) {
        const auto local = rulesp->Load();
        return pkt->L3ACLPort(*local);
    };
}
inline SeparateFunction ACLSeparator(std::shared_ptr<RulesPointer> rulesp) {
    return [rulesp](packet::Packet *pkt) {
        const auto local = rulesp->Load();
        return pkt->L3ACLPermit(*local);
    };
}

// The vector separator of every clone, backed by one shared batcher (engine form).
inline VectorSeparateFunction ACLVectorSeparator(std::shared_ptr<SharedBatcher> batcher) {
    return [batcher](packet::Packet *const *pkts, const bool *mask, bool *answers) {
        const packet::Packet *sel[vBurstSize];
        int idx[vBurstSize];
        size_t n = 0;
        for (int i = 0; i < vBurstSize; ++i) {
            answers[i] = false;
            if (mask[i] && pkts[i]) { sel[n] = pkts[i]; idx[n++] = i; }
        }
        uint32_t ports[vBurstSize] = {0};
        batcher->Classify(sel, n, ports);
        for (size_t k = 0; k < n; ++k) answers[idx[k]] = ports[k] > 0;
    };
}

// The same over a device batcher against the current rule set of `rulesp`
// (step08's pattern in vector form: the pointer is loaded once per burst).
inline VectorSplitFunction ACLVectorSplitter(std::shared_ptr<SharedBatcher> batcher,
                                             std::shared_ptr<RulesPointer> rulesp) {
    return [batcher, rulesp](packet::Packet *const *pkts, const bool *mask, uint8_t *answers) {
        const auto local = rulesp->Load();
        const packet::Packet *sel[vBurstSize];
        int idx[vBurstSize];
        size_t n = 0;
        for (int i = 0; i < vBurstSize; ++i) {
            answers[i] = 0;
            if (mask[i] && pkts[i]) { sel[n] = pkts[i]; idx[n++] = i; }
        }
        uint32_t ports[vBurstSize] = {0};
        batcher->Classify(local.get(), sel, n, ports);
        for (size_t k = 0; k < n; ++k) answers[idx[k]] = static_cast<uint8_t>(ports[k]);
    };
}

// Burst aggregator: bursts are appended into one slot buffer and classified
// in a single GPU call per Flush() (or automatically once `capacity` packets
// are queued); each burst's callback receives its verdicts in order.
class Aggregator {
public:
    using Done = std::function<void(const uint32_t *ports, size_t n)>;
    Aggregator(std::shared_ptr<const packet::L3Rules> rules, size_t capacity = 1 << 20)
        : rules_(std::move(rules)), capacity_(capacity) {
        slots_.reserve(capacity_ * packet::kSlot);
    }
    ~Aggregator() { Flush(); }

    void Push(const packet::Packet *const *pkts, size_t n, Done done) {
        if (queued_ + n > capacity_) Flush();
        slots_.resize((queued_ + n) * packet::kSlot, 0);
        for (size_t i = 0; i < n; ++i) {
            uint8_t *dst = &slots_[(queued_ + i) * packet::kSlot];
            std::memset(dst, 0, packet::kSlot);
            const uint32_t len = pkts[i]->Len < packet::kSlot ? pkts[i]->Len : packet::kSlot;
            if (len) std::memcpy(dst, pkts[i]->Ether, len);
        }
        bursts_.push_back({queued_, n, std::move(done)});
        queued_ += n;
    }

    void Flush() {
        if (queued_ == 0) return;
        std::vector<uint32_t> ports(queued_);
        const int st = nffacl_classify_host(rules_->engine(), slots_.data(), packet::kSlot, queued_,
                                            ports.data(), nullptr);
        if (st != NFFACL_OK) throw std::runtime_error("nffacl_classify_host failed");
        for (auto &b : bursts_) b.done(ports.data() + b.first, b.n);
        bursts_.clear();
        slots_.clear();
        queued_ = 0;
    }

private:
    struct Burst {
        size_t first, n;
        Done done;
    };
    std::shared_ptr<const packet::L3Rules> rules_;
    size_t capacity_;
    size_t queued_ = 0;
    std::vector<uint8_t> slots_;
    std::vector<Burst> bursts_;
};

}  // namespace flow
}  // namespace nffgo
