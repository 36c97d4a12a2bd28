// acl_internal_test.cpp — the reference's packet/acl_internal_test.go restated
// in C++ against the nffgo host mirror (nff-go_amd/host/nffgo.hpp), so the
// parity tests read like the reference's own: same test names, same context
// tables (rulesL3Ctxt, l4Context, l3Context4/6), same cartesian products and
// the same "want outNum iff every field is ok" rule.
//
//   ./acl_internal_test parse   TestGetL3ACLFromJSON, TestGetL3ACLFromTextTable (CPU)
//   ./acl_internal_test match   TestInternal_l4ACL_*, TestInternal_l3ACL_*,
//                               TestInternal_l2ACL_* (GPU: every verdict comes from
//                               libnffacl's HIP kernels)
//   L2: TestGetL2ACLFromJSON / TestGetL2ACLFromTextTable (parse, CPU)
//
// Test packets follow packet/utils_for_test.go:33-126 (InitEmpty*Packet +
// initEtherAddrs/initIPv4Addrs/initIPv6Addrs/initPorts, payload 100 bytes).
#include <unistd.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <atomic>
#include <thread>

#include "nffgo.hpp"

using namespace nffgo;

// ---- minimal go-test style harness ------------------------------------------
struct T {
    const char *name;
    int errors = 0;
    void Errorf(const char *fmt, ...) __attribute__((format(printf, 2, 3))) {
        if (errors++ < 5) {
            va_list ap;
            va_start(ap, fmt);
            std::fprintf(stderr, "    %s: ", name);
            std::vfprintf(stderr, fmt, ap);
            std::fputc('\n', stderr);
            va_end(ap);
        }
    }
};
static int g_failed = 0;
static void run(const char *name, void (*fn)(T &)) {
    T t{name};
    fn(t);
    std::printf("--- %s: %s\n", t.errors ? "FAIL" : "PASS", name);
    if (t.errors) ++g_failed;
}

// ---- rulesL3Ctxt (acl_internal_test.go:91-161) ---------------------------------
struct Addr4Test { const char *raw; uint32_t addr, mask; };
struct Addr6Test { const char *raw; uint8_t addr[16], mask[16]; };
struct IdTest { const char *raw; uint8_t id, mask; };
struct PortTest { const char *raw; uint16_t min, max; bool valid; };
struct RuleTest { const char *raw; uint32_t out; };

static const Addr4Test srcs4[] = {{"ANY", 0x00000000, 0x00000000}, {"127.0.0.1/31", 0x0000007f, 0xfeffffff}};
static const Addr4Test dsts4[] = {{"ANY", 0x00000000, 0x00000000}, {"128.9.9.5/24", 0x00090980, 0x00ffffff}};
static const Addr6Test srcs6[] = {
    {"ANY", {0}, {0}},
    {"::/0", {0}, {0}},
    {"dead::beef/16", {0xde, 0xad}, {0xff, 0xff}},
};
static const Addr6Test dsts6[] = {
    {"ANY", {0}, {0}},
    {"::/0", {0}, {0}},
    {"dead::beef/128", {0xde, 0xad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xbe, 0xef},
     {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff}},
};
static const IdTest ids[] = {{"ANY", 0, 0x00}, {"TCP", 0x06, 0xff}, {"UDP", 0x11, 0xff}, {"ICMP", 0x01, 0xff}};
static const PortTest srcports[] = {{"ANY", 0, 65535, false}, {"1222", 1222, 1222, true}, {"0:222", 0, 222, true}};
static const PortTest dstports[] = {{"ANY", 0, 65535, false}, {"1222", 1222, 1222, true}};
static const RuleTest rules_ctx[] = {{"Accept", 1}, {"Reject", 0}, {"3", 3}, {"", 0}};

struct TestL3Rule {
    std::string SrcAddr, DstAddr, ID, SrcPort, DstPort, OutputNumber;
    bool ipv6;
    nffacl_rule4 want4;
    nffacl_rule6 want6;
};

// generateTestL3Rules (acl_internal_test.go:266-370); orig==true means the
// reference's decisions slice stays nil (its text variant generates nothing),
// so both variants here use decisions = rules[:2] to make the text test real.
static std::vector<TestL3Rule> generateTestL3Rules(bool ipv4, bool ipv6) {
    std::vector<TestL3Rule> table;
    for (int ri = 0; ri < 2; ++ri) {
        const RuleTest &r = rules_ctx[ri];
        for (const IdTest &id : ids)
            for (const PortTest &sport : srcports)
                for (const PortTest &dport : dstports) {
                    if (std::string(id.raw) == "ICMP" && (std::string(sport.raw) != "ANY" || std::string(dport.raw) != "ANY"))
                        continue;  // ICMP rule: both ports must be ANY
                    nffacl_l4 l4{};
                    l4.id = id.id;
                    l4.id_mask = id.mask;
                    l4.valid = (sport.valid || dport.valid) ? 1 : 0;
                    l4.src_port_min = sport.min;
                    l4.src_port_max = sport.max;
                    l4.dst_port_min = dport.min;
                    l4.dst_port_max = dport.max;
                    if (ipv4)
                        for (const Addr4Test &s : srcs4)
                            for (const Addr4Test &d : dsts4) {
                                TestL3Rule t{s.raw, d.raw, id.raw, sport.raw, dport.raw, r.raw, false, {}, {}};
                                t.want4 = nffacl_rule4{r.out, s.addr, d.addr, s.mask, d.mask, l4};
                                table.push_back(t);
                            }
                    if (ipv6)
                        for (const Addr6Test &s : srcs6)
                            for (const Addr6Test &d : dsts6) {
                                TestL3Rule t{s.raw, d.raw, id.raw, sport.raw, dport.raw, r.raw, true, {}, {}};
                                t.want6.output_number = r.out;
                                std::memcpy(t.want6.src_addr, s.addr, 16);
                                std::memcpy(t.want6.dst_addr, d.addr, 16);
                                std::memcpy(t.want6.src_mask, s.mask, 16);
                                std::memcpy(t.want6.dst_mask, d.mask, 16);
                                t.want6.l4 = l4;
                                table.push_back(t);
                            }
                }
    }
    return table;
}

static std::string tmpfile_with(const std::string &content, const char *suffix) {
    char path[] = "/tmp/nffacl_testXXXXXX";
    int fd = mkstemp(path);
    if (fd < 0) std::abort();
    if (write(fd, content.data(), content.size()) != static_cast<ssize_t>(content.size())) std::abort();
    close(fd);
    std::string p = std::string(path) + suffix;
    std::rename(path, p.c_str());
    return p;
}

static bool same4(const nffacl_rule4 &a, const nffacl_rule4 &b) { return std::memcmp(&a, &b, sizeof a) == 0; }
static bool same6(const nffacl_rule6 &a, const nffacl_rule6 &b) { return std::memcmp(&a, &b, sizeof a) == 0; }

static void check_parsed(T &t, const TestL3Rule &r, const packet::RulesOrError &got, const char *what) {
    if (got.second) {
        t.Errorf("%s returned error %s", what, got.second->Error().c_str());
        return;
    }
    if (!r.ipv6) {
        auto v = got.first->ip4();
        if (v.empty() || !same4(v[0], r.want4))
            t.Errorf("Incorrect parse L3 ipv4 rule %s %s %s %s %s %s", r.SrcAddr.c_str(), r.DstAddr.c_str(),
                     r.ID.c_str(), r.SrcPort.c_str(), r.DstPort.c_str(), r.OutputNumber.c_str());
    } else {
        auto v = got.first->ip6();
        if (v.empty() || !same6(v[0], r.want6))
            t.Errorf("Incorrect parse L3 ipv6 rule %s %s %s %s %s %s", r.SrcAddr.c_str(), r.DstAddr.c_str(),
                     r.ID.c_str(), r.SrcPort.c_str(), r.DstPort.c_str(), r.OutputNumber.c_str());
    }
}

// TestGetL3ACLFromJSON (acl_internal_test.go:372-432): json.Marshal(rawL3Rules) -> file -> parse
static void TestGetL3ACLFromJSON(T &t) {
    for (bool v6 : {false, true})
        for (const TestL3Rule &r : generateTestL3Rules(!v6, v6)) {
            std::string doc = "{\"L3Rules\":[{\"SrcAddr\":\"" + r.SrcAddr + "\",\"DstAddr\":\"" + r.DstAddr +
                              "\",\"ID\":\"" + r.ID + "\",\"SrcPort\":\"" + r.SrcPort + "\",\"DstPort\":\"" +
                              r.DstPort + "\",\"OutputNumber\":\"" + r.OutputNumber + "\"}]}";
            const std::string f = tmpfile_with(doc, ".json");
            check_parsed(t, r, packet::GetL3ACLFromJSON(f), "GetL3ACLFromJSON");
            std::remove(f.c_str());
        }
}

// TestGetL3ACLFromTextTable (acl_internal_test.go:434-497) with real cases
static void TestGetL3ACLFromTextTable(T &t) {
    const std::string header =
        "# Source address, Destination address, L4 protocol ID, Source port, Destination port, Output port\n";
    for (bool v6 : {false, true})
        for (const TestL3Rule &r : generateTestL3Rules(!v6, v6)) {
            const std::string line = r.SrcAddr + " " + r.DstAddr + " " + r.ID + " " + r.SrcPort + " " + r.DstPort +
                                     " " + r.OutputNumber;
            const std::string f = tmpfile_with(header + line, ".orig");
            check_parsed(t, r, packet::GetL3ACLFromTextTable(f), "GetL3ACLFromTextTable");
            std::remove(f.c_str());
        }
}

// Error paths keep the reference's codes (common.ErrorCode).
static void TestGetL3ACLErrors(T &t) {
    struct Case { const char *text; common::ErrorCode code; };
    const Case cases[] = {
        {"ANY ANY TCP\n", common::ErrorCode::ParseRuleErr},
        {"ANY ANY SCTP ANY ANY Accept\n", common::ErrorCode::IncorrectArgInRules},
        {"ANY ANY ICMP 1 ANY Accept\n", common::ErrorCode::IncorrectArgInRules},
        {"ANY ANY TCP 9:1 ANY Accept\n", common::ErrorCode::IncorrectArgInRules},
        {"1.2.3.4/8 ::/0 ANY ANY ANY Accept\n", common::ErrorCode::IncorrectArgInRules},
        {"ANY ANY ANY ANY ANY Maybe\n", common::ErrorCode::IncorrectRule},
    };
    for (const Case &c : cases) {
        const std::string f = tmpfile_with(c.text, ".orig");
        auto got = packet::GetL3ACLFromTextTable(f);
        if (!got.second || got.second->Code != c.code) t.Errorf("wrong error for %s", c.text);
        std::remove(f.c_str());
    }
    auto missing = packet::GetL3ACLFromTextTable("/nonexistent/rules.conf");
    if (!missing.second || missing.second->Code != common::ErrorCode::FileErr) t.Errorf("missing file: want FileErr");
    auto badjson = packet::GetL3ACLFromJSON(tmpfile_with("{\"L3Rules\": [", ".json"));
    if (!badjson.second || badjson.second->Code != common::ErrorCode::ParseRuleJSONErr)
        t.Errorf("bad JSON: want ParseRuleJSONErr");
}

// ---- test packets (utils_for_test.go:33-126, packet.go:509-705) ----------------
static const uint8_t kDMAC[6] = {0x00, 0x11, 0x22, 0x33, 0x44, 0x55};
static const uint8_t kSMAC[6] = {0x01, 0x11, 0x21, 0x31, 0x41, 0x51};
static const uint32_t payloadSize = 100;

static std::vector<uint8_t> ether(uint16_t et, size_t total) {
    std::vector<uint8_t> p(total, 0);
    std::memcpy(&p[0], kDMAC, 6);
    std::memcpy(&p[6], kSMAC, 6);
    p[12] = uint8_t(et >> 8);
    p[13] = uint8_t(et);
    return p;
}
static void ports(std::vector<uint8_t> &p, size_t l4) {  // initPorts: 1234 -> 5678
    p[l4] = 1234 >> 8; p[l4 + 1] = 1234 & 255; p[l4 + 2] = 5678 >> 8; p[l4 + 3] = 5678 & 255;
}
static std::vector<uint8_t> ipv4Packet(uint8_t proto, uint32_t l4len, bool withPorts) {
    auto p = ether(types::IPV4Number, types::EtherLen + types::IPv4MinLen + l4len + payloadSize);
    const uint32_t tot = types::IPv4MinLen + l4len + payloadSize;
    p[14] = 0x45; p[16] = uint8_t(tot >> 8); p[17] = uint8_t(tot); p[22] = 64; p[23] = proto;
    const uint8_t src[4] = {127, 0, 0, 1}, dst[4] = {128, 9, 9, 5};
    std::memcpy(&p[26], src, 4);
    std::memcpy(&p[30], dst, 4);
    if (withPorts) ports(p, 34);
    if (proto == types::TCPNumber) p[34 + 12] = 0x50;  // DataOff
    return p;
}
static std::vector<uint8_t> ipv6Packet(uint8_t proto, uint32_t l4len, bool withPorts) {
    auto p = ether(types::IPV6Number, types::EtherLen + types::IPv6Len + l4len + payloadSize);
    p[14] = 0x60;  // VtcFlow
    const uint32_t pl = l4len + payloadSize;
    p[18] = uint8_t(pl >> 8); p[19] = uint8_t(pl); p[20] = proto; p[21] = 255;
    const uint8_t a[16] = {0xde, 0xad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xbe, 0xaf};  // dead::beaf
    std::memcpy(&p[22], a, 16);
    std::memcpy(&p[38], a, 16);
    if (withPorts) ports(p, 54);
    if (proto == types::TCPNumber) p[54 + 12] = 0x50;
    return p;
}

struct TestPacket {
    std::vector<uint8_t> bytes;
    packet::Packet pkt() const { return packet::Packet{bytes.data(), static_cast<uint32_t>(bytes.size())}; }
};
static TestPacket getIPv4TCPTestPacket() { return {ipv4Packet(types::TCPNumber, types::TCPMinLen, true)}; }
static TestPacket getIPv4ICMPTestPacket() { return {ipv4Packet(types::ICMPNumber, types::ICMPLen, false)}; }
static TestPacket getIPv6TCPTestPacket() { return {ipv6Packet(types::TCPNumber, types::TCPMinLen, true)}; }
static TestPacket getIPv6UDPTestPacket() { return {ipv6Packet(types::UDPNumber, types::UDPLen, true)}; }
static TestPacket getIPv6ICMPTestPacket() { return {ipv6Packet(types::ICMPv6Number, types::ICMPLen, false)}; }

// l3ACL of one packet against a one-rule L3Rules literal
static uint32_t l3ACL(const TestPacket &tp, const std::vector<nffacl_rule4> &ip4, const std::vector<nffacl_rule6> &ip6) {
    auto rules = packet::L3Rules::FromRecords(ip4, ip6);
    return tp.pkt().L3ACLPort(*rules);
}

// ---- contexts of the match tests --------------------------------------------------
struct PortRange { uint16_t min, max; bool valid, ok; };
struct IDMask { uint8_t id, mask; bool ok; };
struct Addr4Mask { uint32_t addr, msk; bool ok; };
struct Addr6Mask { uint8_t addr[16], msk[16]; bool ok; };

static const Addr4Mask srcAddrMsk4[] = {{0x0100007f, 0xffffffff, true}, {0, 0, true}, {0x0200007f, 0x00ffffff, true},
                                        {0x0200007f, 0xffffffff, false}};
static const Addr4Mask dstAddrMsk4[] = {{0x05090980, 0xffffffff, true}, {0, 0, true}, {0x0200007f, 0x00ffffff, false},
                                        {0x05050980, 0x0000ffff, true}};
static const Addr6Mask addrMsk6[] = {
    {{0}, {0}, true},
    {{0xde, 0xad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xbb, 0xbb}, {0xff, 0xff, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xff, 0xff}, false},
    {{0xde, 0xad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xdd, 0xdd}, {0xff, 0xff}, true},
};

// TestInternal_l4ACL_packetIPv4_TCP (:501-537): l4ACL alone — here through
// l3ACL with an ANY rule whose L4 has valid=true and OutputNumber 1.
static void TestInternal_l4ACL_packetIPv4_TCP(T &t) {
    const TestPacket pkt = getIPv4TCPTestPacket();
    const PortRange srcRange[] = {{0, 65535, true, true}, {1234, 1234, true, true}, {1233, 1299, true, true},
                                  {0, 0, true, false}, {2000, 2000, true, false}};
    const PortRange dstRange[] = {{0, 65535, true, true}, {5678, 5678, true, true}, {9999, 9999, true, false}};
    for (const auto &s : srcRange)
        for (const auto &d : dstRange) {
            nffacl_rule4 r{};
            r.output_number = 1;
            r.l4 = nffacl_l4{0, 0, 1, 0, s.min, s.max, d.min, d.max};
            const bool got = l3ACL(pkt, {r}, {}) == 1;
            if (got != (s.ok && d.ok)) t.Errorf("rule (%u-%u, %u-%u): got %d", s.min, s.max, d.min, d.max, got);
        }
}

// TestInternal_l3ACL_packetIPv4_TCP (:540-610)
static void TestInternal_l3ACL_packetIPv4_TCP(T &t) {
    const TestPacket pkt = getIPv4TCPTestPacket();
    for (uint32_t outNum : {0u, 1u, 10u, 65535u})
        for (const auto &s : srcAddrMsk4)
            for (const auto &d : dstAddrMsk4) {
                nffacl_rule4 r{};
                r.output_number = outNum;
                r.src_addr = s.addr; r.dst_addr = d.addr; r.src_mask = s.msk; r.dst_mask = d.msk;
                const uint32_t want = (s.ok && d.ok) ? outNum : 0;
                const uint32_t got = l3ACL(pkt, {r}, {});
                if (got != want) t.Errorf("out %u src %08x/%08x dst %08x/%08x: got %u want %u", outNum, s.addr, s.msk,
                                          d.addr, d.msk, got, want);
            }
}

template <bool V6, size_t NI, size_t NS, size_t ND, size_t NA>
static void l3l4(T &t, const TestPacket &pkt, const IDMask (&idMsk)[NI], const PortRange (&srcRange)[NS],
                 const PortRange (&dstRange)[ND], const void *addrs, size_t nsrc) {
    (void)NA;
    for (const auto &id : idMsk)
        for (const auto &s : srcRange)
            for (const auto &d : dstRange) {
                const nffacl_l4 l4{id.id, id.mask, static_cast<uint8_t>(s.valid || d.valid), 0, s.min, s.max, d.min, d.max};
                for (uint32_t outNum : {0u, 1u, 65535u}) {
                    if (!V6) {
                        for (const auto &sa : srcAddrMsk4)
                            for (const auto &da : dstAddrMsk4) {
                                const nffacl_rule4 r{outNum, sa.addr, da.addr, sa.msk, da.msk, l4};
                                const uint32_t want = (id.ok && s.ok && d.ok && sa.ok && da.ok) ? outNum : 0;
                                const uint32_t got = l3ACL(pkt, {r}, {});
                                if (got != want) t.Errorf("id %u sp %u-%u dp %u-%u out %u: got %u want %u", id.id, s.min,
                                                          s.max, d.min, d.max, outNum, got, want);
                            }
                    } else {
                        const Addr6Mask *a6 = static_cast<const Addr6Mask *>(addrs);
                        for (size_t i = 0; i < nsrc; ++i)
                            for (size_t j = 0; j < nsrc; ++j) {
                                nffacl_rule6 r{};
                                r.output_number = outNum;
                                std::memcpy(r.src_addr, a6[i].addr, 16);
                                std::memcpy(r.src_mask, a6[i].msk, 16);
                                std::memcpy(r.dst_addr, a6[j].addr, 16);
                                std::memcpy(r.dst_mask, a6[j].msk, 16);
                                r.l4 = l4;
                                const uint32_t want = (id.ok && s.ok && d.ok && a6[i].ok && a6[j].ok) ? outNum : 0;
                                const uint32_t got = l3ACL(pkt, {}, {r});
                                if (got != want) t.Errorf("v6 id %u sp %u-%u dp %u-%u out %u: got %u want %u", id.id,
                                                          s.min, s.max, d.min, d.max, outNum, got, want);
                            }
                    }
                }
            }
}

static const PortRange kSrcTU[] = {{0, 65535, false, true}, {13, 17, true, false}, {1234, 1234, true, true},
                                   {1233, 1299, true, true}, {0, 0, true, false}};
static const PortRange kDstTU[] = {{0, 65535, false, true}, {9999, 9999, true, false}, {5678, 5678, true, true}};
static const PortRange kSrcICMP[] = {{0, 65535, false, true}, {13, 17, true, false}, {1234, 1234, true, false}};
static const PortRange kDstICMP[] = {{0, 65535, false, true}, {9999, 9999, true, false}, {5678, 5678, true, false}};

static void TestInternal_l3ACL_l4ACL_packetIPv4_TCP(T &t) {  // :612-703
    const IDMask id[] = {{0, 0, true}, {6, 0xff, true}, {17, 0xff, false}};
    l3l4<false, 3, 5, 3, 0>(t, getIPv4TCPTestPacket(), id, kSrcTU, kDstTU, nullptr, 0);
}
static void TestInternal_l3ACL_l4ACL_packetIPv6_TCP(T &t) {  // :706-819
    const IDMask id[] = {{0, 0, true}, {6, 0xff, true}, {17, 0xff, false}};
    l3l4<true, 3, 5, 3, 0>(t, getIPv6TCPTestPacket(), id, kSrcTU, kDstTU, addrMsk6, 3);
}
static void TestInternal_l3ACL_l4ACL_packetIPv6_UDP(T &t) {  // :822-935
    const IDMask id[] = {{0, 0, true}, {6, 0xff, false}, {17, 0xff, true}};
    l3l4<true, 3, 5, 3, 0>(t, getIPv6UDPTestPacket(), id, kSrcTU, kDstTU, addrMsk6, 3);
}
static void TestInternal_l3ACL_l4ACL_packetIPv4_ICMP(T &t) {  // :937-1027
    const IDMask id[] = {{0, 0, true}, {6, 0xff, false}, {17, 0xff, false}, {1, 0xff, true}};
    l3l4<false, 4, 3, 3, 0>(t, getIPv4ICMPTestPacket(), id, kSrcICMP, kDstICMP, nullptr, 0);
}
static void TestInternal_l3ACL_l4ACL_packetIPv6_ICMP(T &t) {  // :1029-1141
    const IDMask id[] = {{0, 0, true}, {6, 0xff, false}, {17, 0xff, false}, {58, 0xff, true}};
    l3l4<true, 4, 3, 3, 0>(t, getIPv6ICMPTestPacket(), id, kSrcICMP, kDstICMP, addrMsk6, 3);
}

// Vector separator / splitter over the stability-test rule files
// (testSingleWorkingFF.go:404-451, 532-560): ports 111/222/333 round robin.
static void TestVectorSeparatorStability(T &t) {
    const char *dir = std::getenv("NFFACL_GOLDEN");
    const std::string g = dir ? dir : "tests/golden";
    auto sep = packet::GetL3ACLFromTextTable(g + "/rules/test-separate-l3rules.conf");
    auto spl = packet::GetL3ACLFromTextTable(g + "/rules/test-split.conf");
    if (sep.second || spl.second) { t.Errorf("cannot load stability rule files"); return; }
    std::vector<TestPacket> tp;
    for (int i = 0; i < flow::vBurstSize; ++i) {
        TestPacket p{ipv4Packet(types::UDPNumber, types::UDPLen, true)};
        const uint16_t dport = (i % 3 == 0) ? 111 : (i % 3 == 1) ? 222 : 333;
        p.bytes[36] = uint8_t(dport >> 8);
        p.bytes[37] = uint8_t(dport);
        tp.push_back(p);
    }
    std::vector<packet::Packet> pk;
    for (auto &p : tp) pk.push_back(p.pkt());
    packet::Packet *ptrs[flow::vBurstSize];
    bool mask[flow::vBurstSize], answers[flow::vBurstSize] = {false};
    uint8_t outs[flow::vBurstSize] = {0};
    for (int i = 0; i < flow::vBurstSize; ++i) { ptrs[i] = &pk[i]; mask[i] = i != 5; }
    flow::ACLVectorSeparator(sep.first)(ptrs, mask, answers);
    flow::ACLVectorSplitter(spl.first)(ptrs, mask, outs);
    for (int i = 0; i < flow::vBurstSize; ++i) {
        const bool want = mask[i] && i % 3 == 0;
        if (answers[i] != want) t.Errorf("separator lane %d: got %d", i, answers[i]);
        const uint8_t wout = mask[i] ? uint8_t(i % 3 + 1) : 0;
        if (outs[i] != wout) t.Errorf("splitter lane %d: got %u want %u", i, outs[i], wout);
    }
    // Aggregator: two bursts, one GPU call
    flow::Aggregator agg(sep.first);
    std::vector<uint32_t> got;
    const packet::Packet *cp[flow::vBurstSize];
    for (int i = 0; i < flow::vBurstSize; ++i) cp[i] = &pk[i];
    for (int b = 0; b < 2; ++b)
        agg.Push(cp, flow::vBurstSize, [&](const uint32_t *p, size_t n) { got.insert(got.end(), p, p + n); });
    agg.Flush();
    for (size_t i = 0; i < got.size(); ++i)
        if ((got[i] != 0) != (i % flow::vBurstSize % 3 == 0)) t.Errorf("aggregator packet %zu: got %u", i, got[i]);
    if (got.size() != 2 * flow::vBurstSize) t.Errorf("aggregator returned %zu verdicts", got.size());
}

// ---- L2 (acl_internal_test.go:66-89, 174-273, 1144-1273) -------------------------
struct MacAddrTest { const char *raw; uint8_t addr[6]; bool notAny; };
struct IdTest16 { const char *raw; uint16_t id, mask; };
static const MacAddrTest l2srcs[] = {{"ANY", {0}, false}, {"00:11:22:33:44:55", {0x00, 0x11, 0x22, 0x33, 0x44, 0x55}, true}};
static const MacAddrTest l2dsts[] = {{"ANY", {0}, false}, {"01:11:21:31:41:51", {0x01, 0x11, 0x21, 0x31, 0x41, 0x51}, true}};
static const IdTest16 l2ids[] = {{"ANY", 0, 0}, {"IPv4", 0x0800, 0xffff}, {"IPv6", 0x86dd, 0xffff}, {"arp", 0x0806, 0xffff}};

struct TestL2Rule { std::string Rule, Source, Destination, ID; nffacl_l2_rule want; };

// generateTestL2Rules (:174-213); `orig` uses all four decisions (the
// reference's text variant iterates a nil slice and tests nothing).
static std::vector<TestL2Rule> generateTestL2Rules(bool orig) {
    std::vector<TestL2Rule> table;
    const int nd = orig ? 4 : 2;
    for (int ri = 0; ri < nd; ++ri)
        for (const MacAddrTest &src : l2srcs)
            for (const MacAddrTest &dst : l2dsts)
                for (const IdTest16 &id : l2ids) {
                    nffacl_l2_rule w{};
                    w.output_number = rules_ctx[ri].out;
                    w.daddr_not_any = dst.notAny;
                    w.saddr_not_any = src.notAny;
                    std::memcpy(w.daddr, dst.addr, 6);
                    std::memcpy(w.saddr, src.addr, 6);
                    w.id_mask = id.mask;
                    w.id = id.id;
                    table.push_back(TestL2Rule{rules_ctx[ri].raw, src.raw, dst.raw, id.raw, w});
                }
    return table;
}

static void check_l2(T &t, const TestL2Rule &r, const packet::L2RulesOrError &got, const char *what) {
    if (got.second) {
        t.Errorf("%s returned error %s", what, got.second->Error().c_str());
        return;
    }
    auto v = got.first->eth();
    if (v.empty() || std::memcmp(&v[0], &r.want, sizeof r.want) != 0)
        t.Errorf("Incorrect parse L2 rule %s %s %s %s", r.Source.c_str(), r.Destination.c_str(), r.ID.c_str(),
                 r.Rule.c_str());
}

// TestGetL2ACLFromJSON (:217-243)
static void TestGetL2ACLFromJSON(T &t) {
    for (const TestL2Rule &r : generateTestL2Rules(false)) {
        const std::string doc = "{\"L2Rules\":[{\"Rule\":\"" + r.Rule + "\",\"Source\":\"" + r.Source +
                                "\",\"Destination\":\"" + r.Destination + "\",\"ID\":\"" + r.ID + "\"}]}";
        const std::string f = tmpfile_with(doc, ".json");
        check_l2(t, r, packet::GetL2ACLFromJSON(f), "GetL2ACLFromJSON");
        std::remove(f.c_str());
    }
}

// TestGetL2ACLFromTextTable (:247-273)
static void TestGetL2ACLFromTextTable(T &t) {
    for (const TestL2Rule &r : generateTestL2Rules(true)) {
        const std::string text = "# Source MAC, Destination MAC, L3 ID, Output port\n" + r.Source + " " +
                                 r.Destination + " " + r.ID + " " + r.Rule;
        const std::string f = tmpfile_with(text, ".orig");
        check_l2(t, r, packet::GetL2ACLFromTextTable(f), "GetL2ACLFromTextTable");
        std::remove(f.c_str());
    }
}

struct MacAddr { uint8_t addr[6]; bool notAny, ok; };
struct IDMask16 { uint16_t id, mask; bool ok; };

// getARPRequestTestPacket (utils_for_test.go:95-104 -> arp.go:79-93)
static std::vector<uint8_t> arpRequestPacket() {
    std::vector<uint8_t> p(types::EtherLen + 28, 0);
    std::memset(&p[0], 0xff, 6);
    std::memcpy(&p[6], kSMAC, 6);
    p[12] = 0x08; p[13] = 0x06;
    const uint8_t hdr[8] = {0, 1, 0x08, 0x00, 6, 4, 0, 1};  // HType, PType, HLen, PLen, Operation
    std::memcpy(&p[14], hdr, 8);
    std::memcpy(&p[22], kSMAC, 6);
    const uint8_t spa[4] = {127, 0, 0, 1}, tpa[4] = {128, 9, 9, 5};
    std::memcpy(&p[28], spa, 4);
    std::memset(&p[32], 0xff, 6);
    std::memcpy(&p[38], tpa, 4);
    return p;
}

static void l2Table(T &t, const std::vector<uint8_t> &frame, const IDMask16 (&idMsk)[4], const MacAddr (&srcMac)[3],
                    const MacAddr (&dstMac)[3]) {
    packet::Packet pkt{frame.data(), static_cast<uint32_t>(frame.size())};
    const uint32_t outs[] = {0, 1, 65535};
    for (uint32_t outNum : outs)
        for (const IDMask16 &im : idMsk)
            for (const MacAddr &src : srcMac)
                for (const MacAddr &dst : dstMac) {
                    nffacl_l2_rule r{};
                    r.output_number = outNum;
                    r.saddr_not_any = src.notAny;
                    r.daddr_not_any = dst.notAny;
                    std::memcpy(r.saddr, src.addr, 6);
                    std::memcpy(r.daddr, dst.addr, 6);
                    r.id_mask = im.mask;
                    r.id = im.id;
                    auto rules = packet::L2Rules::FromRecords({r});
                    const uint32_t got = pkt.L2ACLPort(*rules);
                    const uint32_t want = (im.ok && src.ok && dst.ok) ? outNum : 0;
                    if (got != want) t.Errorf("Incorrect result for rule out=%u id=%04x: got %u want %u", outNum, im.id, got, want);
                }
}

// TestInternal_l2ACL_packetIPv4 (:1144-1207)
static void TestInternal_l2ACL_packetIPv4(T &t) {
    const IDMask16 idMsk[4] = {{0, 0, true}, {0x0800, 0xffff, true}, {0x86dd, 0xffff, false}, {0x0806, 0xffff, false}};
    const MacAddr srcMac[3] = {{{0}, false, true}, {{0x01, 0x11, 0x21, 0x31, 0x41, 0x51}, true, true},
                               {{0, 0x55, 0x55, 0x55, 0x55, 0}, true, false}};
    const MacAddr dstMac[3] = {{{0}, false, true}, {{0x00, 0x11, 0x22, 0x33, 0x44, 0x55}, true, true},
                               {{0x01, 0x11, 0x21, 0x31, 0x41, 0x51}, true, false}};
    l2Table(t, ipv4Packet(types::UDPNumber, types::UDPLen, true), idMsk, srcMac, dstMac);
}

// TestInternal_l2ACL_packetARP (:1209-1273)
static void TestInternal_l2ACL_packetARP(T &t) {
    const IDMask16 idMsk[4] = {{0, 0, true}, {0x0800, 0xffff, false}, {0x86dd, 0xffff, false}, {0x0806, 0xffff, true}};
    const MacAddr srcMac[3] = {{{0}, false, true}, {{0x01, 0x11, 0x21, 0x31, 0x41, 0x51}, true, true},
                               {{0x0, 0x11, 0x22, 0x33, 0x44, 0x55}, true, false}};
    const MacAddr dstMac[3] = {{{0}, false, true}, {{0xff, 0xff, 0xff, 0xff, 0xff, 0xff}, true, true},
                               {{0x01, 0x11, 0x21, 0x31, 0x41, 0x51}, true, false}};
    l2Table(t, arpRequestPacket(), idMsk, srcMac, dstMac);
}

// Many flow-function clones (threads) sharing one batcher: every burst's
// answers must equal the single-clone separator's (acl.go semantics).
static void TestVectorSeparatorSharedBatcher(T &t) {
    const char *dir = std::getenv("NFFACL_GOLDEN");
    const std::string g = dir ? dir : "tests/golden";
    auto sep = packet::GetL3ACLFromTextTable(g + "/rules/test-separate-l3rules.conf");
    if (sep.second) { t.Errorf("cannot load rules"); return; }
    std::vector<TestPacket> tp;
    for (int i = 0; i < flow::vBurstSize; ++i) {
        TestPacket p{ipv4Packet(types::UDPNumber, types::UDPLen, true)};
        const uint16_t dport = (i % 3 == 0) ? 111 : (i % 3 == 1) ? 222 : 333;
        p.bytes[36] = uint8_t(dport >> 8);
        p.bytes[37] = uint8_t(dport);
        tp.push_back(p);
    }
    std::vector<packet::Packet> pk;
    for (auto &p : tp) pk.push_back(p.pkt());
    auto batcher = std::make_shared<flow::SharedBatcher>(sep.first, 4096, 50, 4);
    auto fn = flow::ACLVectorSeparator(batcher);
    constexpr int kClones = 8, kBursts = 200;
    std::atomic<int> bad{0};
    std::vector<std::thread> clones;
    for (int c = 0; c < kClones; ++c)
        clones.emplace_back([&, c] {
            packet::Packet *ptrs[flow::vBurstSize];
            bool mask[flow::vBurstSize], answers[flow::vBurstSize];
            for (int b = 0; b < kBursts; ++b) {
                for (int i = 0; i < flow::vBurstSize; ++i) {
                    ptrs[i] = &pk[i];
                    mask[i] = ((i + b + c) % 5) != 0;
                }
                fn(ptrs, mask, answers);
                for (int i = 0; i < flow::vBurstSize; ++i)
                    if (answers[i] != (mask[i] && i % 3 == 0)) ++bad;
            }
        });
    for (auto &th : clones) th.join();
    const auto st = batcher->Stats();
    if (bad) t.Errorf("%d wrong answers", bad.load());
    if (st.bursts != uint64_t(kClones) * kBursts) t.Errorf("bursts %llu", (unsigned long long)st.bursts);
    if (st.batches >= st.bursts) t.Errorf("no aggregation: %llu batches for %llu bursts",
                                          (unsigned long long)st.batches, (unsigned long long)st.bursts);
}

// SetSeparator's scalar call shape (firewall.go:54-57, flow.go:128): clones
// classifying one packet per call through the GPU's persistent consumer;
// every answer must be the single-packet verdict.
static void TestScalarSeparatorService(T &t) {
    const char *dir = std::getenv("NFFACL_GOLDEN");
    const std::string g = dir ? dir : "tests/golden";
    auto split = packet::GetL3ACLFromTextTable(g + "/rules/test-split.conf");
    if (split.second) { t.Errorf("cannot load rules"); return; }
    std::vector<TestPacket> tp;
    for (int i = 0; i < 3; ++i) {
        TestPacket p{ipv4Packet(types::UDPNumber, types::UDPLen, true)};
        const uint16_t dport = i == 0 ? 111 : i == 1 ? 222 : 333;
        p.bytes[36] = uint8_t(dport >> 8);
        p.bytes[37] = uint8_t(dport);
        tp.push_back(p);
    }
    std::vector<packet::Packet> pk;
    for (auto &p : tp) pk.push_back(p.pkt());
    auto sep = flow::ACLSeparator(split.first);
    auto spl = flow::ACLSplitter(split.first);
    constexpr int kClones = 16, kCalls = 400;
    std::atomic<int> bad{0};
    std::vector<std::thread> clones;
    for (int c = 0; c < kClones; ++c)
        clones.emplace_back([&, c] {
            for (int k = 0; k < kCalls; ++k) {
                const int i = (k + c) % 3;
                if (spl(&pk[i]) != uint32_t(i + 1)) ++bad;  // test-split.conf: 111 -> 1, 222 -> 2, 333 -> 3
                if (!sep(&pk[i])) ++bad;
            }
        });
    for (auto &th : clones) th.join();
    if (bad) t.Errorf("%d wrong answers", bad.load());
}

// examples/tutorial/step08.go replayed: a reload thread loads a new rule file
// every few ms (GetL3ACLFromTextTable) and swaps the pointer atomically
// (step08.go:38-44) while 16 clones classify — one 32-packet burst through
// the shared device batcher and one scalar L3ACLPort per iteration — each
// against the rule set it loaded (step08.go:33-35).  Generation k maps dst
// ports 111/222/333 to outputs rotated by k and port 444 to 10 + k, so every
// answer names the rule set that produced it.
static void TestRuleReloadStep08(T &t) {
    struct Gen {
        std::shared_ptr<const packet::L3Rules> rules;
        int k;
    };
    auto load_gen = [&](int k) -> std::shared_ptr<const Gen> {
        std::string text;
        const int dp[4] = {111, 222, 333, 444};
        for (int i = 0; i < 4; ++i)
            text += "ANY ANY ANY ANY " + std::to_string(dp[i]) + " " +
                    std::to_string(i < 3 ? (i + k) % 3 + 1 : 10 + k) + "\n";
        const std::string path = tmpfile_with(text, ".conf");
        auto r = packet::GetL3ACLFromTextTable(path);
        std::remove(path.c_str());
        if (r.second) return nullptr;
        r.first->Prepare();  // compile + upload in the reload thread, not in a clone's call
        return std::make_shared<const Gen>(Gen{r.first, k});
    };
    auto expect = [](int k, int i) -> uint32_t { return i < 3 ? uint32_t((i + k) % 3 + 1) : uint32_t(10 + k); };
    std::vector<TestPacket> tp;
    for (int i = 0; i < 4; ++i) {
        TestPacket p{ipv4Packet(types::UDPNumber, types::UDPLen, true)};
        const uint16_t dport = i == 0 ? 111 : i == 1 ? 222 : i == 2 ? 333 : 444;
        p.bytes[36] = uint8_t(dport >> 8);
        p.bytes[37] = uint8_t(dport);
        tp.push_back(p);
    }
    std::vector<packet::Packet> pk;
    for (auto &p : tp) pk.push_back(p.pkt());
    std::shared_ptr<const Gen> cur = load_gen(0);
    if (!cur) { t.Errorf("cannot load generation 0"); return; }
    auto batcher = std::make_shared<flow::SharedBatcher>(-1, 4096, 50, 4);
    constexpr int kClones = 16, kReloads = 40;
    std::atomic<bool> halt{false};
    std::atomic<int> bad{0}, bursts{0};
    std::vector<std::atomic<int>> seen(kReloads + 1);
    std::vector<std::thread> clones;
    for (int c = 0; c < kClones; ++c)
        clones.emplace_back([&, c] {
            const packet::Packet *burst[flow::vBurstSize];
            int which[flow::vBurstSize];
            uint32_t ports[flow::vBurstSize];
            for (int it = 0; !halt.load(); ++it) {
                const std::shared_ptr<const Gen> local = std::atomic_load(&cur);  // atomic.LoadPointer
                for (int i = 0; i < flow::vBurstSize; ++i) {
                    which[i] = (i + it + c) % 4;
                    burst[i] = &pk[which[i]];
                }
                batcher->Classify(local->rules.get(), burst, flow::vBurstSize, ports);
                for (int i = 0; i < flow::vBurstSize; ++i)
                    if (ports[i] != expect(local->k, which[i])) ++bad;
                // the same burst as one request to the resident consumer (burst mailbox)
                packet::L3ACLPortBurst(burst, flow::vBurstSize, ports, *local->rules);
                for (int i = 0; i < flow::vBurstSize; ++i)
                    if (ports[i] != expect(local->k, which[i])) ++bad;
                const int i = (it + c) % 4;
                if (pk[i].L3ACLPort(*local->rules) != expect(local->k, i)) ++bad;
                ++seen[local->k];
                ++bursts;
            }
        });
    for (int k = 1; k <= kReloads; ++k) {  // updateSeparateRules, time.Sleep shortened
        std::this_thread::sleep_for(std::chrono::milliseconds(3));
        auto next = load_gen(k);
        if (!next) { t.Errorf("cannot load generation %d", k); break; }
        std::atomic_store(&cur, next);  // atomic.StorePointer; the old set frees with its last user
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(3));
    halt = true;
    for (auto &th : clones) th.join();
    int gens = 0;
    for (auto &s : seen) gens += s.load() > 0;
    if (bad) t.Errorf("%d answers from the wrong rule set", bad.load());
    if (gens < kReloads / 2) t.Errorf("only %d of %d generations were classified against", gens, kReloads + 1);
    const auto st = batcher->Stats();
    if (st.bursts < uint64_t(bursts.load())) t.Errorf("batcher saw %llu bursts", (unsigned long long)st.bursts);
}

int main(int argc, char **argv) {
    const std::string which = argc > 1 ? argv[1] : "parse";
    if (which == "parse" || which == "all") {
        run("TestGetL3ACLFromJSON", TestGetL3ACLFromJSON);
        run("TestGetL3ACLFromTextTable", TestGetL3ACLFromTextTable);
        run("TestGetL3ACLErrors", TestGetL3ACLErrors);
        run("TestGetL2ACLFromJSON", TestGetL2ACLFromJSON);
        run("TestGetL2ACLFromTextTable", TestGetL2ACLFromTextTable);
    }
    if (which == "match" || which == "all") {
        run("TestInternal_l4ACL_packetIPv4_TCP", TestInternal_l4ACL_packetIPv4_TCP);
        run("TestInternal_l3ACL_packetIPv4_TCP", TestInternal_l3ACL_packetIPv4_TCP);
        run("TestInternal_l3ACL_l4ACL_packetIPv4_TCP", TestInternal_l3ACL_l4ACL_packetIPv4_TCP);
        run("TestInternal_l3ACL_l4ACL_packetIPv6_TCP", TestInternal_l3ACL_l4ACL_packetIPv6_TCP);
        run("TestInternal_l3ACL_l4ACL_packetIPv6_UDP", TestInternal_l3ACL_l4ACL_packetIPv6_UDP);
        run("TestInternal_l3ACL_l4ACL_packetIPv4_ICMP", TestInternal_l3ACL_l4ACL_packetIPv4_ICMP);
        run("TestInternal_l3ACL_l4ACL_packetIPv6_ICMP", TestInternal_l3ACL_l4ACL_packetIPv6_ICMP);
        run("TestVectorSeparatorStability", TestVectorSeparatorStability);
        run("TestInternal_l2ACL_packetIPv4", TestInternal_l2ACL_packetIPv4);
        run("TestInternal_l2ACL_packetARP", TestInternal_l2ACL_packetARP);
        run("TestVectorSeparatorSharedBatcher", TestVectorSeparatorSharedBatcher);
        run("TestScalarSeparatorService", TestScalarSeparatorService);
        run("TestRuleReloadStep08", TestRuleReloadStep08);
    }
    std::printf(g_failed ? "FAIL\n" : "ok\n");
    return g_failed ? 1 : 0;
}
