// compile.hpp — host-side compilation of an nffacl_rules set into the device
// table blob (internal to libnffacl).
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "rules.hpp"
#include "table.hpp"

namespace nffacl {

// One key dimension ("slot") of the indexed table of a family (table.hpp).
struct DimInfo {
    uint32_t kind = 0;       // KeyKind
    uint32_t shift = 0;      // bucket = key >> shift (1-D)
    uint32_t kind2 = kKeyNone;  // 2-D slots: bucket = (key >> shift) << bits2 | key2 >> shift2
    uint32_t shift2 = 0, bits2 = 0;
    uint32_t n_buckets = 0;  // 2^(key bits - shift)
    uint32_t off_dir = 0;    // dword offset of dir[n_buckets + 1] (or, with off_dir16, of the
                             // 2-level directory's group bases base[n_buckets / 64 + 2])
    uint32_t off_dir16 = 0;  // 0, or dword offset of the u16 offsets dir16[n_buckets + 1]:
                             // dir[t] = base[t >> 6] + dir16[t]
    uint32_t dir8 = 0;       // 1: off_dir16 holds u8 offsets instead, dir[t] = base[t >> 4] + dir8[t];
                             // 2: 4-bit bucket counts, dir[t] = base[t >> 4] + sum(cnt[16 (t >> 4) .. t - 1])
    uint32_t off_ent = 0;    // dword offset of the bucket entries (inline rule entries)
    uint32_t n_rules = 0;    // rules assigned to this dimension
    uint64_t n_ent = 0;      // bucket entries (with replication)
    uint32_t max_list = 0;   // longest bucket list
};

// Indexed view of one address family.  INDEXED and the LDS-directory HYBRID
// forms: 4 slots in the order [dst address, src address, dst port, src port]
// (empty slots allowed).  HYBRID global-directory form: up to kMaxSlots
// slots of any 1-D / 2-D key, all non-empty.
struct FamilyIndex {
    uint32_t entry_dwords = 0;  // INDEXED / lane form: 8 (IPv4) or 20 (IPv6); flat forms 6 / 12
    uint32_t off_ent_base = 0;  // flat forms: dword offset of the family's first entry (directory values count from it)
    DimInfo dims[kMaxSlots];
    uint32_t off_resid = 0, n_resid = 0;  // residual entries (scanned linearly)
    uint32_t used_slots = 0;              // 1 + last non-empty slot (kernels walk that many)
};

struct CompiledTable {
    int algo = NFFACL_ALGO_LINEAR;
    // One contiguous blob of dwords, uploaded as is.
    std::vector<uint32_t> blob;
    // LINEAR: rule records (dword offsets into blob) and live record counts.
    uint32_t off_rec4 = 0, n4 = 0;
    uint32_t off_rec6 = 0, n6 = 0;
    // INDEXED / HYBRID: per family key slots + residual entries.
    // HYBRID: off_rec4/off_rec6 = the cold records; blob[0, lds_dwords) = the
    // directories staged in LDS.
    FamilyIndex idx4, idx6;
    uint32_t lds_dwords = 0;
    // HYBRID flat-LDS: rounds of candidate loads in flight (2 or 4)
    uint32_t flat_rounds = 2;
    // flat-LDS walk with many expected candidates per packet: its entry
    // loads are issued without a per-lane branch (engine.hip kTabFlatLds4U)
    uint32_t flat_uncond = 0;
    // no rule constrains a port (every record's port bounds are [0, 65535]
    // both ways): the INDEXED LDS kernel skips the L4 port extraction and
    // tests (engine.hip kTabLdsNP)
    uint32_t ports_any = 0;
    // two-level LDS directories with u8 offsets per 16-bucket group (every
    // slot of the table; DimInfo::dir8)
    uint32_t dir8 = 0;
    // HYBRID global-directory form with generalized slots (dims[k].kind2 etc.;
    // idx*.used_slots = slots in use, all non-empty)
    bool slots_g = false;
    uint32_t off_empty_dir = 0;  // slots_g: dword offset of an empty directory {0, 0}
    uint32_t off_params = 0;     // flat-LDS positional forms: the slot parameter block (table.hpp kFlatParams), 0 = none
};

// Table-layout overrides for tuning experiments (unset in production).
struct CompileOptions {
    int flat = 2;           // NFFACL_TUNE_FLAT: HYBRID form 0 lane, 1 flat (global dirs), 2 flat-LDS
    size_t dir_bytes = 0;   // NFFACL_TUNE_DIR_KB: HYBRID directory budget (0 = policy)
    int slots2d = 1;        // NFFACL_TUNE_SLOTS2D: global-directory form may use 2-D slots;
                            // 2: flat-LDS with generalized 1-D / 2-D slots
    double slot_cost = 0.1; // NFFACL_TUNE_SLOT_COST (1/100): expected candidates per packet a slot must save
    bool dir16 = true;      // NFFACL_TUNE_DIR16: two-level u16 LDS directories allowed
    bool dir8 = true;       // NFFACL_TUNE_DIR8: two-level u8 LDS directories allowed (HYBRID)
    bool dir4 = true;       // NFFACL_TUNE_DIR4: two-level 4-bit-count LDS directories allowed (flat-LDS
                            // positional forms, when they buy finer radixes: table.hpp kDir4GroupShift)
    int uncond = -1;        // NFFACL_TUNE_UNCOND: flat-LDS branch-free entry loads (-1 = policy)
    // NFFACL_TUNE_FINE_A / _P: fine 2-D address x port slots of the flat-LDS
    // form (positional slots 4..7), a address bits x p port bits; a = 0: none
    int fine_a = 9;          // address bits of the fine grids: 9 with the 4-bit directories (C5 0.4941 vs
                             // 0.5128 ms at 8: a third fewer 1-D entries, 3.9 vs 5.0 MB; profiles/r5_ab/fine/);
                             // round 4, u8 directories: 8 x 4 on slots 4-5 0.583 vs 0.626 (profiles/r4_ab/fine/)
    int fine_p = 5;          // 8 x 5: C5 0.5741 / 0.5718 vs 0.5829 / 0.5825 ms in two sweeps (ab_c5_fine_sweep*)
    double fine_gain = 0.5;  // NFFACL_TUNE_FINE_G (1/100): a rule moves below this fraction of its 1-D cover
    int fine_min = 256;      // NFFACL_TUNE_FINE_MIN: fewest moved rules worth a fine slot
    int fine_slots = 3;      // NFFACL_TUNE_FINE_SLOTS: bit k allows fine slot 4 + k (3: dst x dport, src x dport)
    int cgrid = 0;           // NFFACL_TUNE_CGRID: coarse address grids on free positional slots 6 / 7: the
                             // dst / src slot's rules replicated into >= 2^cgrid buckets move to a grid of
                             // radix rb - cgrid (same candidates, far fewer copies: a smaller, L2-resident table)
    int dir_sbias = 0;       // NFFACL_TUNE_DIR_SB (percent): weight of the size-biased list length (the lists
                             // traffic that matches rules lands in) beside the uniform-key mean in the radix sizing
    int dir_per_rule = 16;   // NFFACL_TUNE_DIR_PER_RULE: LDS directory buckets per rule before the budget cut
                             // (C3 0.4005 vs 0.4122 ms at 4: profiles/r4_ab/fine/ab_c3_dir_per_rule.json)
    bool coarse = false;    // NFFACL_TUNE_COARSE: flat-LDS coarse address slots for short prefixes
                            // (C5 table 7.7 -> 3.7 MB but 0.722 vs 0.649 ms: off; profiles/r2_dir8/coarse/)
    // false (+ `err`) if a set variable is out of range
    static bool from_env(CompileOptions &o, std::string &err);
};

// Integer environment variable in [lo, hi]: false (+ `err`) if set but
// malformed or out of range; `set` says whether it was set.
bool env_knob(const char *name, long lo, long hi, long &v, bool &set, std::string &err);

// Compile `rules`.  algo: NFFACL_ALGO_LINEAR, _INDEXED, _HYBRID or AUTO.
bool compile_table(const nffacl_rules &rules, int algo, const CompileOptions &opt, CompiledTable &out,
                   std::string &err);

}  // namespace nffacl
