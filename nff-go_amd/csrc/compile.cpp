// compile.cpp — turns a parsed rule set (acl.go's ip4/ip6 slices) into the
// device table blob described in table.hpp.
//
// Semantics preserved from packet/acl.go:522-565 and :508-520:
//  * first match in slice order per family, Reject (OutputNumber 0) included;
//  * IPv4 rules test ports only when l4.valid (acl.go:535-540);
//  * IPv6 rules ALWAYS test ports (acl.go:555-558), whatever l4.valid says;
//  * the port test is min <= port <= max per direction, so a rule whose
//    tested range is empty (min > max, possible only for records built
//    directly, never from the parsers) can never match and is dropped here.
#include "compile.hpp"

#include <cstring>

namespace nffacl {

namespace {

uint32_t le32(const uint8_t *b) {
    return uint32_t(b[0]) | uint32_t(b[1]) << 8 | uint32_t(b[2]) << 16 | uint32_t(b[3]) << 24;
}

bool emit_rec4(const nffacl_rule4 &r, std::vector<uint32_t> &out) {
    const bool port_check = r.l4.valid != 0;
    if (port_check && (r.l4.src_port_min > r.l4.src_port_max || r.l4.dst_port_min > r.l4.dst_port_max))
        return false;  // l4ACL can never pass
    uint32_t lo = 0, hi = 0xFFFFFFFFu;
    if (port_check) {
        lo = uint32_t(r.l4.src_port_min) | uint32_t(r.l4.dst_port_min) << 16;
        hi = uint32_t(r.l4.src_port_max) | uint32_t(r.l4.dst_port_max) << 16;
    }
    const bool full = lo == 0 && hi == 0xFFFFFFFFu;
    out.push_back(r.src_addr);
    out.push_back(r.src_mask);
    out.push_back(r.dst_addr);
    out.push_back(r.dst_mask);
    out.push_back(uint32_t(r.l4.id) | uint32_t(r.l4.id_mask) << 8 | (full ? 0u : kMetaPortCheck));
    out.push_back(lo);
    out.push_back(hi);
    out.push_back(r.output_number);
    return true;
}

bool emit_rec6(const nffacl_rule6 &r, std::vector<uint32_t> &out) {
    if (r.l4.src_port_min > r.l4.src_port_max || r.l4.dst_port_min > r.l4.dst_port_max) return false;
    const uint32_t lo = uint32_t(r.l4.src_port_min) | uint32_t(r.l4.dst_port_min) << 16;
    const uint32_t hi = uint32_t(r.l4.src_port_max) | uint32_t(r.l4.dst_port_max) << 16;
    const bool full = lo == 0 && hi == 0xFFFFFFFFu;
    for (int k = 0; k < 4; ++k) out.push_back(le32(r.src_addr + 4 * k));
    for (int k = 0; k < 4; ++k) out.push_back(le32(r.src_mask + 4 * k));
    for (int k = 0; k < 4; ++k) out.push_back(le32(r.dst_addr + 4 * k));
    for (int k = 0; k < 4; ++k) out.push_back(le32(r.dst_mask + 4 * k));
    out.push_back(uint32_t(r.l4.id) | uint32_t(r.l4.id_mask) << 8 | (full ? 0u : kMetaPortCheck));
    out.push_back(lo);
    out.push_back(hi);
    out.push_back(r.output_number);
    return true;
}

}  // namespace

bool compile_table(const nffacl_rules &rules, int algo, CompiledTable &out, std::string &err) {
    if (algo != NFFACL_ALGO_AUTO && algo != NFFACL_ALGO_LINEAR && algo != NFFACL_ALGO_INDEXED) {
        err = "unknown algorithm";
        return false;
    }
    out = CompiledTable{};
    std::vector<uint32_t> rec4, rec6;
    rec4.reserve(rules.ip4.size() * kRec4Dwords);
    rec6.reserve(rules.ip6.size() * kRec6Dwords);
    for (const auto &r : rules.ip4)
        if (emit_rec4(r, rec4)) ++out.n4;
    for (const auto &r : rules.ip6)
        if (emit_rec6(r, rec6)) ++out.n6;
    out.off_rec4 = 0;
    out.off_rec6 = static_cast<uint32_t>(rec4.size());
    out.blob = std::move(rec4);
    out.blob.insert(out.blob.end(), rec6.begin(), rec6.end());
    out.algo = NFFACL_ALGO_LINEAR;
    if (out.blob.empty()) out.blob.push_back(0);  // keep a valid allocation
    return true;
}

}  // namespace nffacl
