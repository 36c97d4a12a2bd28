// compile.hpp — host-side compilation of an nffacl_rules set into the device
// table blob (internal to libnffacl).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rules.hpp"
#include "table.hpp"

namespace nffacl {

struct CompiledTable {
    int algo = NFFACL_ALGO_LINEAR;
    // One contiguous blob of dwords, uploaded as is.
    std::vector<uint32_t> blob;
    // Linear records (dword offsets into blob) and live record counts.
    uint32_t off_rec4 = 0, n4 = 0;
    uint32_t off_rec6 = 0, n6 = 0;
    // Indexed: per family, dimension headers (dword offsets into blob),
    // plus the residual list (records not covered by any dimension).
    uint32_t n_dims4 = 0, off_dims4 = 0;
    uint32_t n_dims6 = 0, off_dims6 = 0;
    uint32_t off_resid4 = 0, n_resid4 = 0;
    uint32_t off_resid6 = 0, n_resid6 = 0;
    // Stats for reporting.
    uint64_t max_list4 = 0, max_list6 = 0;
    double mean_list4 = 0.0, mean_list6 = 0.0;
};

// Compile `rules`.  algo: NFFACL_ALGO_LINEAR, NFFACL_ALGO_INDEXED or AUTO.
bool compile_table(const nffacl_rules &rules, int algo, CompiledTable &out, std::string &err);

}  // namespace nffacl
