// compile.hpp — host-side compilation of an nffacl_rules set into the device
// table blob (internal to libnffacl).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rules.hpp"
#include "table.hpp"

namespace nffacl {

// One key dimension of the indexed table (see table.hpp).
struct DimInfo {
    uint32_t kind = 0;       // KeyKind
    uint32_t shift = 0;      // bucket = key >> shift
    uint32_t n_buckets = 0;  // 2^(key bits - shift)
    uint32_t off_dir = 0, off_cands = 0;  // dword offsets into blob
    uint32_t n_rules = 0;    // rules assigned to this dimension
    uint64_t n_cands = 0;    // total candidate entries (with replication)
    uint32_t max_list = 0;   // longest bucket list
};

// Indexed view of one address family.
struct FamilyIndex {
    uint32_t n_dims = 0;
    DimInfo dims[4];
    uint32_t off_resid = 0, n_resid = 0;  // residual record indices (scanned linearly)
};

struct CompiledTable {
    int algo = NFFACL_ALGO_LINEAR;
    // One contiguous blob of dwords, uploaded as is.
    std::vector<uint32_t> blob;
    // Linear records (dword offsets into blob) and live record counts.
    uint32_t off_rec4 = 0, n4 = 0;
    uint32_t off_rec6 = 0, n6 = 0;
    // Indexed: per family key dimensions + residual list.
    FamilyIndex idx4, idx6;
};

// Compile `rules`.  algo: NFFACL_ALGO_LINEAR, NFFACL_ALGO_INDEXED or AUTO.
bool compile_table(const nffacl_rules &rules, int algo, CompiledTable &out, std::string &err);

}  // namespace nffacl
