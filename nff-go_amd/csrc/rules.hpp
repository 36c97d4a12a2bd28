// rules.hpp — host-side rule set of libnffacl (internal).
//
// nffacl_rules is the C-ABI handle for the reference's *packet.L3Rules
// (packet/acl.go:451-455): two ordered slices, one per address family, in the
// order the rule file lists them.  Records keep the reference's field meaning
// exactly (see include/nffacl.h); the device compiler (compile.cpp) derives its
// own layouts from them.
#pragma once

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "nffacl.h"

namespace nffacl {
struct DevTable;                  // engine.hpp
constexpr int kMaxDevices = 16;   // HIP devices a rule set can be compiled for
}  // namespace nffacl

struct nffacl_rules {
    std::vector<nffacl_rule4> ip4;
    std::vector<nffacl_rule6> ip6;
    // The compiled device table of this rule set, one per HIP device, built
    // on first use by the calls that take the rule set itself (the scalar
    // service, per-burst batcher submits, nffacl_rules_prepare) and retired
    // with it in nffacl_rules_free: the Go binding's *L3Rules owns its table,
    // so a rule reload (examples/tutorial/step08.go:38-44) is "load the new
    // rules, store the pointer" exactly as in the reference.  Published once
    // (release) and immutable afterwards; readers load without a lock.
    mutable std::atomic<nffacl::DevTable *> dev[nffacl::kMaxDevices] = {};
    mutable std::mutex dev_mu;  // serialises the first compile per device
};

struct nffacl_l2rules {
    std::vector<nffacl_l2_rule> eth;  // L2Rules.eth, acl.go:457-460
};

namespace nffacl {

// Compiled table of `rules` on HIP device `dev` (built + uploaded on first
// use; service.hip).  nullptr + status on failure.
DevTable *rules_table(const nffacl_rules *rules, int dev, int &status);
// Retire every device table of `rules` (nffacl_rules_free).
void release_rules_tables(const nffacl_rules *rules);

// One line of a rule file after field splitting: acl.go:55-62 rawL3Rule.
struct RawL3Rule {
    std::string src_addr, dst_addr, id, src_port, dst_port, output_number;
};

struct ParseError {
    int code = NFFACL_OK;  // negated common.ErrorCode
    std::string message;
};

// rawL3Parse (acl.go:226-355).  Appends to `out`; returns false and fills
// `err` at the first bad rule.
bool raw_l3_parse(const std::vector<RawL3Rule> &raw, nffacl_rules &out, ParseError &err);

// GetL3ACLFromTextTable body (acl.go:156-177) over an in-memory file image.
bool parse_text_table(const char *data, size_t len, nffacl_rules &out, ParseError &err);

// GetL3ACLFromJSON body (acl.go:129-133) over an in-memory file image.
bool parse_json(const char *data, size_t len, nffacl_rules &out, ParseError &err);

// rawL2Rule (acl.go:44-49).
struct RawL2Rule {
    std::string rule, source, destination, id;
};

// rawL2Parse (acl.go:356-383), GetL2ACLFromTextTable body (acl.go:97-117),
// GetL2ACLFromJSON body (acl.go:78-83).
bool raw_l2_parse(const std::vector<RawL2Rule> &raw, nffacl_l2rules &out, ParseError &err);
bool parse_l2_text_table(const char *data, size_t len, nffacl_l2rules &out, ParseError &err);
bool parse_l2_json(const char *data, size_t len, nffacl_l2rules &out, ParseError &err);

// go1.13 net.ParseMAC (6-, 8- or 20-byte hardware addresses).
bool go_parse_mac(const std::string &s, std::vector<uint8_t> &hw);

// go1.13 net.ParseCIDR restricted to what rawL3Parse consumes: the masked
// network address (4 bytes for dotted-quad input, 16 for IPv6 syntax) and the
// mask.  Returns false where Go returns an error.
bool go_parse_cidr(const std::string &s, std::vector<uint8_t> &ip, std::vector<uint8_t> &mask);

// go1.13 strings.Fields (unicode.IsSpace separators).
std::vector<std::string> go_fields(const std::string &line);

// go1.13 strconv.ParseUint(s, 10, bits).
bool go_parse_uint10(const std::string &s, int bits, uint64_t &out);

}  // namespace nffacl
