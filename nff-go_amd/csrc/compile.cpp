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

#include <algorithm>
#include <cmath>
#include <array>
#include <cstdlib>
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

// ---------------------------------------------------------------------------
// Indexed table
// ---------------------------------------------------------------------------

namespace {

uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

uint32_t lead_ones(uint32_t m) { return m == 0xFFFFFFFFu ? 32u : static_cast<uint32_t>(__builtin_clz(~m)); }

struct KeyRange {
    uint32_t lo, hi;  // inclusive, in key space
    double cover;     // fraction of the key domain
};

// Superset interval of an address constraint (addr ^ x) & mask == 0 on the
// big-endian key: the leading-ones run of the mask is a prefix, so the
// matching set is inside [a & p, (a & p) | ~p].
KeyRange addr_range(uint32_t addr_le, uint32_t mask_le) {
    const uint32_t a = bswap32(addr_le), m = bswap32(mask_le);
    const uint32_t L = lead_ones(m);
    const uint32_t p = L == 0 ? 0u : (0xFFFFFFFFu << (32 - L));
    return KeyRange{a & p, (a & p) | ~p, std::ldexp(1.0, -static_cast<int>(L))};
}

KeyRange port_range(uint32_t mn, uint32_t mx) {
    return KeyRange{mn, mx, (double(mx) - double(mn) + 1.0) / 65536.0};
}

// Key ranges of record r in dimension order [dst, src, dport, sport].
void rec_ranges(const uint32_t *rec, bool v6, KeyRange out[4]) {
    const uint32_t *m = v6 ? rec + 16 : rec + 4;  // meta, lo, hi
    if (v6) {
        out[0] = addr_range(rec[8], rec[12]);
        out[1] = addr_range(rec[0], rec[4]);
    } else {
        out[0] = addr_range(rec[2], rec[3]);
        out[1] = addr_range(rec[0], rec[1]);
    }
    const bool pc = (m[0] & kMetaPortCheck) != 0;
    const uint32_t lo = pc ? m[1] : 0u, hi = pc ? m[2] : 0xFFFFFFFFu;
    out[2] = port_range(lo >> 16, hi >> 16);
    out[3] = port_range(lo & 0xFFFFu, hi & 0xFFFFu);
}

struct DimBuild {
    uint32_t kind = 0;
    uint32_t key_bits = 32;
    // fine 2-D slot (flat-LDS positional slots 4..7, build_hybrid): bucket =
    // (key >> shift) << bits2 | key2 >> shift2; lists filled by GSlot::fill
    uint32_t kind2 = kKeyNone, shift2 = 0, bits2 = 0;
    std::vector<uint32_t> rules;  // record indices, ascending
    std::vector<KeyRange> ranges; // parallel to rules
    // built
    uint32_t rb = 0, shift = 0, max_list = 0;
    uint32_t max_rb = 32;             // radix cap (coarse address slots, see build_hybrid)
    std::vector<uint32_t> dir, ents;  // ents: record indices per bucket entry
    std::vector<uint64_t> span;       // per rule: buckets covered
};

// Radix bits for a dimension holding n rules: about 4 buckets per rule,
// at most 2^20 buckets (addresses) / 2^16 (ports, i.e. one bucket per port).
uint32_t pick_rb(size_t n, uint32_t key_bits, size_t per_rule = 4) {
    uint32_t rb = 4;
    while (rb < 20 && (size_t(1) << rb) < per_rule * n) ++rb;
    return std::min(rb, key_bits);
}

uint64_t budget_for(size_t n) { return 8ull * n + 65536ull; }

// Coarse address slots (build_hybrid): rules kCoarseGap+ bits shorter than
// their slot's radix move, when the slot holds >= kCoarseMinRules rules and
// >= kCoarseMinMoved of them would move.
constexpr uint32_t kCoarseGap = 3;
constexpr size_t kCoarseMinRules = 4096;
constexpr size_t kCoarseMinMoved = 256;

// Fewest rules worth a source-port slot of their own (see assign_family).
constexpr size_t kMinSportRules = 128;

// Fine 2-D slots (build_hybrid): a family needs kFineMinRules rules (and a
// slot CompileOptions::fine_min moved rules).
constexpr uint32_t kFineMinRules = 4096;

// Pick the radix width and count the replicated entries of the dimension's
// bucket lists: start at ~4 buckets per rule and narrow the radix while wide
// rules would replicate past the budget.
uint64_t span_dim(DimBuild &d) {
    uint64_t total = 0;
    for (uint32_t rb = pick_rb(d.rules.size(), d.key_bits);; --rb) {
        d.rb = rb;
        d.shift = d.key_bits - rb;
        d.span.assign(d.rules.size(), 0);
        total = 0;
        for (size_t i = 0; i < d.rules.size(); ++i) {
            d.span[i] = uint64_t(d.ranges[i].hi >> d.shift) - (d.ranges[i].lo >> d.shift) + 1;
            total += d.span[i];
        }
        if (total <= budget_for(d.rules.size()) || rb <= 4) break;
    }
    return total;
}

// Bucket t holds, in ascending rule order, every rule whose key range meets
// [t << shift, ((t+1) << shift) - 1]; dir[t] .. dir[t+1] delimit it.
void finish_dim(DimBuild &d) {
    if (d.rules.empty()) {  // empty slot: 2 empty buckets
        d.rb = 1;
        d.shift = d.key_bits - 1;
        d.dir.assign(3, 0);
        d.ents.clear();
        d.max_list = 0;
        return;
    }
    span_dim(d);
    const size_t nb = size_t(1) << d.rb;
    std::vector<uint32_t> len(nb + 1, 0);
    for (const KeyRange &r : d.ranges)
        for (uint64_t t = r.lo >> d.shift; t <= (r.hi >> d.shift); ++t) ++len[t];
    d.dir.assign(nb + 1, 0);
    d.max_list = 0;
    for (size_t t = 0; t < nb; ++t) {
        d.dir[t + 1] = d.dir[t] + len[t];
        d.max_list = std::max(d.max_list, len[t]);
    }
    d.ents.assign(d.dir[nb], 0);
    std::vector<uint32_t> fill(d.dir.begin(), d.dir.end() - 1);
    for (size_t i = 0; i < d.rules.size(); ++i)  // ascending rule order -> sorted lists
        for (uint64_t t = d.ranges[i].lo >> d.shift; t <= (d.ranges[i].hi >> d.shift); ++t)
            d.ents[fill[t]++] = d.rules[i];
}

// Inline entry of record r (table.hpp) appended to blob.
void emit_entry(const uint32_t *rec, bool v6, uint32_t r, std::vector<uint32_t> &blob) {
    if (!v6) {
        const uint32_t meta = rec[4];
        const uint32_t exact = ((meta >> 8) & 0xFFu) ? kEntExact : 0u;
        blob.insert(blob.end(), {rec[0], rec[1], rec[2], rec[3],
                                 (meta & 0xFFu) | exact | (r << kEntIndexShift), rec[5], rec[6], rec[7]});
    } else {
        const uint32_t meta = rec[16];
        const uint32_t exact = ((meta >> 8) & 0xFFu) ? kEntExact : 0u;
        blob.insert(blob.end(), {rec[0], rec[4], rec[8], rec[12],
                                 (meta & 0xFFu) | exact | (r << kEntIndexShift), rec[17], rec[18], rec[19],
                                 rec[1], rec[2], rec[3], rec[5], rec[6], rec[7],
                                 rec[9], rec[10], rec[11], rec[13], rec[14], rec[15]});
    }
}

// Assign the live records of one family to key slots: each rule goes to the
// slot where its key range covers the least of the key domain; past a slot's
// replication budget the widest rules move to their next-best slot (or to the
// residual scan, choice -1).
struct FamilyPlan {
    DimBuild dims[4];
    std::vector<uint32_t> resid;
    std::vector<std::array<KeyRange, 4>> rr;
};

void assign_family(const std::vector<uint32_t> &recs, uint32_t rw, bool v6, uint32_t n, FamilyPlan &plan) {
    static const uint32_t kinds4[4] = {kKeyDst4, kKeySrc4, kKeyDport, kKeySport};
    static const uint32_t kinds6[4] = {kKeyDst6, kKeySrc6, kKeyDport, kKeySport};
    DimBuild *dims = plan.dims;
    auto &rr = plan.rr;
    rr.assign(n, {});
    for (int k = 0; k < 4; ++k) {
        dims[k].kind = v6 ? kinds6[k] : kinds4[k];
        dims[k].key_bits = k < 2 ? 32 : 16;
    }
    // preference order per rule: slots by increasing coverage
    std::vector<int> choice(n, -1);
    std::vector<std::array<int, 4>> pref(n);
    for (uint32_t r = 0; r < n; ++r) {
        KeyRange kr[4];
        rec_ranges(recs.data() + size_t(r) * rw, v6, kr);
        for (int k = 0; k < 4; ++k) rr[r][k] = kr[k];
        std::array<int, 4> o = {0, 1, 2, 3};
        std::stable_sort(o.begin(), o.end(), [&](int a, int b) { return kr[a].cover < kr[b].cover; });
        pref[r] = o;
        choice[r] = kr[o[0]].cover < 1.0 ? o[0] : -1;
    }
    std::vector<int> rank(n, 0);
    // A sparsely used source-port slot costs every packet a directory lookup
    // for few candidates: its rules move to their next-best slot, and the
    // kernels then run with three slots.
    size_t n_sport = 0;
    for (uint32_t r = 0; r < n; ++r) n_sport += choice[r] == 3;
    const bool no_sport = n_sport > 0 && n_sport < std::max<size_t>(kMinSportRules, n / 256);
    if (no_sport) {
        for (uint32_t r = 0; r < n; ++r) {
            if (choice[r] != 3) continue;
            int next = -1;
            while (++rank[r] < 4) {
                const int cand = pref[r][rank[r]];
                if (cand != 3 && rr[r][cand].cover < 1.0) { next = cand; break; }
            }
            choice[r] = next;
        }
    }
    // Bound replication: a slot may hold at most `budget` entries; past it,
    // the widest rules move to their next-best slot (or to the residual scan).
    for (int round = 0; round < 8; ++round) {
        for (int k = 0; k < 4; ++k) {
            dims[k].rules.clear();
            dims[k].ranges.clear();
        }
        for (uint32_t r = 0; r < n; ++r)
            if (choice[r] >= 0) {
                dims[choice[r]].rules.push_back(r);
                dims[choice[r]].ranges.push_back(rr[r][choice[r]]);
            }
        bool moved = false;
        for (int k = 0; k < 4; ++k) {
            DimBuild &d = dims[k];
            if (d.rules.empty()) continue;
            const uint64_t total = span_dim(d);
            const uint64_t budget = budget_for(d.rules.size());
            if (total <= budget) continue;
            std::vector<size_t> idx(d.rules.size());
            for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
            std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return d.span[a] > d.span[b]; });
            uint64_t t = total;
            for (size_t q = 0; q < idx.size() && t > budget; ++q) {
                const uint32_t r = d.rules[idx[q]];
                t -= d.span[idx[q]];
                int next = -1;
                while (++rank[r] < 4) {
                    const int cand = pref[r][rank[r]];
                    if (rr[r][cand].cover < 1.0 && !(no_sport && cand == 3)) { next = cand; break; }
                }
                choice[r] = next;
                moved = true;
            }
        }
        if (!moved) break;
    }
    plan.resid.clear();
    for (uint32_t r = 0; r < n; ++r)
        if (choice[r] < 0) plan.resid.push_back(r);
}

// INDEXED: emit the slots' directories + inline entries and the residual entries.
void build_family(const std::vector<uint32_t> &recs, uint32_t rw, bool v6, uint32_t n,
                  std::vector<uint32_t> &blob, FamilyIndex &fi) {
    FamilyPlan plan;
    assign_family(recs, rw, v6, n, plan);
    const uint32_t ew = v6 ? kEnt6Dwords : kEnt4Dwords;
    fi.entry_dwords = ew;
    for (int k = 0; k < 4; ++k) {
        DimBuild &d = plan.dims[k];
        finish_dim(d);
        DimInfo &di = fi.dims[k];
        di.kind = d.kind;
        di.shift = d.shift;
        di.n_buckets = 1u << d.rb;
        di.n_rules = static_cast<uint32_t>(d.rules.size());
        di.n_ent = d.ents.size();
        di.max_list = d.max_list;
        di.off_dir = static_cast<uint32_t>(blob.size());
        blob.insert(blob.end(), d.dir.begin(), d.dir.end());
        while (blob.size() % 4) blob.push_back(0);  // entries 16-byte aligned
        di.off_ent = static_cast<uint32_t>(blob.size());
        for (uint32_t r : d.ents) emit_entry(recs.data() + size_t(r) * rw, v6, r, blob);
        if (d.ents.empty()) blob.insert(blob.end(), ew, 0u);  // keep entry 0 addressable
        if (!d.rules.empty()) fi.used_slots = k + 1;
    }
    fi.off_resid = static_cast<uint32_t>(blob.size());
    fi.n_resid = static_cast<uint32_t>(plan.resid.size());
    for (uint32_t r : plan.resid) emit_entry(recs.data() + size_t(r) * rw, v6, r, blob);
    while (blob.size() % 4) blob.push_back(0);
}

// ---------------------------------------------------------------------------
// Hybrid table (table.hpp): directories sized to an LDS budget, compact
// 16-byte candidate entries + per-rule cold records in global memory.
// ---------------------------------------------------------------------------

// A big-endian mask is a prefix iff its complement is 0...01...1.
bool prefix32(uint32_t m_be) {
    const uint32_t c = ~m_be;
    return (c & (c + 1u)) == 0u;
}

// Prefix length of a 16-byte wire-order mask, or -1 if it is not a prefix.
int prefix128(const uint32_t *m_le) {
    int len = 0;
    bool ended = false;
    for (int k = 0; k < 4; ++k) {
        const uint32_t w = bswap32(m_le[k]);
        if (ended) {
            if (w) return -1;
            continue;
        }
        if (!prefix32(w)) return -1;
        const int l = __builtin_popcount(w);
        len += l;
        if (l < 32) ended = true;
    }
    return len;
}

// Rules the compact format encodes exactly: CIDR masks (what both parsers
// produce) and id_mask in {0, 0xff}.
bool hybrid_encodable(const std::vector<uint32_t> &rec4, uint32_t n4, const std::vector<uint32_t> &rec6,
                      uint32_t n6) {
    if (n4 >= kMaxIndexedRules || n6 >= kMaxIndexedRules) return false;
    for (uint32_t r = 0; r < n4; ++r) {
        const uint32_t *R = rec4.data() + size_t(r) * kRec4Dwords;
        const uint32_t idm = (R[4] >> 8) & 0xFFu;
        if ((idm != 0 && idm != 0xFF) || !prefix32(bswap32(R[1])) || !prefix32(bswap32(R[3]))) return false;
    }
    for (uint32_t r = 0; r < n6; ++r) {
        const uint32_t *R = rec6.data() + size_t(r) * kRec6Dwords;
        const uint32_t idm = (R[16] >> 8) & 0xFFu;
        if ((idm != 0 && idm != 0xFF) || prefix128(R + 4) < 0 || prefix128(R + 12) < 0) return false;
    }
    return true;
}

// Exact flat-form entry of record r (table.hpp, "flat-form list entry"):
// IPv4 6 dwords, IPv6 12.
void emit_hyb_entry(const uint32_t *rec, bool v6, uint32_t r, std::vector<uint32_t> &blob) {
    const uint32_t *m = v6 ? rec + 16 : rec + 4;  // meta, lo, hi
    uint32_t sl, dl;
    if (v6) {
        sl = static_cast<uint32_t>(prefix128(rec + 4));
        dl = static_cast<uint32_t>(prefix128(rec + 12));
    } else {
        sl = static_cast<uint32_t>(__builtin_popcount(rec[1]));
        dl = static_cast<uint32_t>(__builtin_popcount(rec[3]));
    }
    const bool pc = (m[0] & kMetaPortCheck) != 0;
    const uint32_t lo = pc ? m[1] : 0u, hi = pc ? m[2] : 0xFFFFFFFFu;
    const uint32_t exact = ((m[0] >> 8) & 0xFFu) ? kEntExact : 0u;
    const uint32_t output = v6 ? rec[19] : rec[7];
    const uint32_t ocode = std::min(output, kHybOutEscape);
    const uint32_t sa = v6 ? rec[0] : rec[0], da = v6 ? rec[8] : rec[2];
    blob.insert(blob.end(), {bswap32(sa), bswap32(da), (m[0] & 0xFFu) | exact | (r << kEntIndexShift), lo, hi,
                             sl | dl << 8 | ocode << kHybOutShift});
    if (v6)
        blob.insert(blob.end(), {bswap32(rec[1]), bswap32(rec[2]), bswap32(rec[3]),
                                 bswap32(rec[9]), bswap32(rec[10]), bswap32(rec[11])});
}

// Output number of record r (the family's output array).
void emit_cold(const uint32_t *rec, bool v6, std::vector<uint32_t> &blob) { blob.push_back(v6 ? rec[19] : rec[7]); }

uint64_t entries_at(const DimBuild &d, uint32_t rb) {
    const uint32_t shift = d.key_bits - rb;
    uint64_t total = 0;
    for (const KeyRange &r : d.ranges) total += uint64_t(r.hi >> shift) - (r.lo >> shift) + 1;
    return total;
}

// Radix widths of all eight slots (both families) so that their directories
// fit `budget` bytes: start every slot at ~4 buckets per rule, then narrow,
// one bit at a time, the slot whose mean list grows least per byte saved
// (weighted by its family's share of the rules, a proxy for its share of
// the traffic).
// LDS bytes of a directory of nb buckets in form fmt: 0 plain u32, 16 two-level
// u16 (groups of 64), 8 two-level u8 (groups of 16).
double dir_form_bytes(double nb, int fmt) {
    if (fmt == 4) return 0.5 * (nb + 16) + 8 + 4.0 * (std::floor(nb / (1u << kDir4GroupShift)) + 2);
    if (fmt == 8) return 1.0 * (nb + 8) + 4.0 * (std::floor(nb / (1u << kDir8GroupShift)) + 2);
    if (fmt == 16) return 2.0 * (nb + 4) + 4.0 * (std::floor(nb / (1u << kDir16GroupShift)) + 2);
    return 4.0 * (nb + 1);
}

// LDS directories start at `per_rule` buckets per rule (then narrow to the budget).
thread_local size_t g_dir_per_rule = 4;  // CompileOptions::dir_per_rule of this thread's compile (compile_table)
thread_local double g_dir_sbias = 0.0;   // CompileOptions::dir_sbias / 100

// Size-biased mean list length of a slot at radix b: sum(len^2) / sum(len),
// the list a key drawn like the rules' own keys lands in (traffic that
// matches rules), where the uniform-key mean (entries / buckets) is the list
// of a random key.
double size_biased_at(const DimBuild &d, uint32_t b) {
    const uint32_t shift = d.key_bits - b;
    const size_t nb = size_t(1) << b;
    std::vector<int32_t> diff(nb + 1, 0);
    for (const KeyRange &r : d.ranges) {
        ++diff[r.lo >> shift];
        --diff[size_t(r.hi >> shift) + 1];
    }
    double s1 = 0, s2 = 0;
    int64_t c = 0;
    for (size_t t = 0; t < nb; ++t) {
        c += diff[t];
        s1 += double(c);
        s2 += double(c) * double(c);
    }
    return s1 > 0 ? s2 / s1 : 0.0;
}

void size_directories(DimBuild *const *all, const double *weight, int nd, size_t budget, int fmt) {
    std::vector<uint32_t> rb(nd);
    std::vector<std::vector<double>> mean(nd);
    auto bytes = [&](int i, uint32_t b) {
        if (all[i]->rules.empty()) return 16.0;
        return dir_form_bytes(double(1u << b), fmt);
    };
    for (int i = 0; i < nd; ++i) {
        const DimBuild &d = *all[i];
        if (d.rules.empty()) { rb[i] = 1; continue; }
        rb[i] = std::max(1u, std::min(pick_rb(d.rules.size(), d.key_bits, g_dir_per_rule), d.max_rb));
        mean[i].assign(rb[i] + 1, 0.0);
        for (uint32_t b = 1; b <= rb[i]; ++b) {
            mean[i][b] = double(entries_at(d, b)) / double(1u << b);
            if (g_dir_sbias > 0) mean[i][b] = (1.0 - g_dir_sbias) * mean[i][b] + g_dir_sbias * size_biased_at(d, b);
        }
    }
    double total = 0;
    for (int i = 0; i < nd; ++i) total += bytes(i, rb[i]);
    while (total > double(budget)) {
        int best = -1;
        double best_cost = 0;
        for (int i = 0; i < nd; ++i) {
            if (all[i]->rules.empty() || rb[i] <= 1) continue;
            const double saved = bytes(i, rb[i]) - bytes(i, rb[i] - 1);
            const double cost = weight[i] * (mean[i][rb[i] - 1] - mean[i][rb[i]]) / saved;
            if (best < 0 || cost < best_cost) { best = i; best_cost = cost; }
        }
        if (best < 0) break;
        total -= bytes(best, rb[best]) - bytes(best, rb[best] - 1);
        --rb[best];
    }
    for (int i = 0; i < nd; ++i) {
        DimBuild &d = *all[i];
        d.rb = rb[i];
        d.shift = d.key_bits - rb[i];
    }
}

// Bucket lists of a slot at its chosen radix width (ascending rule order).
void fill_lists(DimBuild &d) {
    const size_t nb = size_t(1) << d.rb;
    std::vector<uint32_t> len(nb, 0);
    for (const KeyRange &r : d.ranges)
        for (uint64_t t = r.lo >> d.shift; t <= (r.hi >> d.shift); ++t) ++len[t];
    d.dir.assign(nb + 1, 0);
    d.max_list = 0;
    for (size_t t = 0; t < nb; ++t) {
        d.dir[t + 1] = d.dir[t] + len[t];
        d.max_list = std::max(d.max_list, len[t]);
    }
    d.ents.assign(d.dir[nb], 0);
    std::vector<uint32_t> fill(d.dir.begin(), d.dir.end() - 1);
    for (size_t i = 0; i < d.rules.size(); ++i)
        for (uint64_t t = d.ranges[i].lo >> d.shift; t <= (d.ranges[i].hi >> d.shift); ++t)
            d.ents[fill[t]++] = d.rules[i];
}

// Radix widths for `budget` bytes of directories, then the bucket lists;
// returns the expected candidates per packet (mean list length summed over
// the slots, families weighted by their share of the rules).
double size_and_fill(DimBuild *const *all, const double *weight, size_t budget, int fmt = 0, int nd = 8) {
    size_directories(all, weight, nd, budget, fmt);
    double expect = 0;
    for (int i = 0; i < nd; ++i) {
        DimBuild &d = *all[i];
        if (d.rules.empty()) {
            d.rb = 1;
            d.shift = d.key_bits - 1;
            d.dir.assign(3, 0);
            d.ents.clear();
            d.max_list = 0;
        } else {
            fill_lists(d);
            expect += weight[i] * double(d.ents.size()) / double(size_t(1) << d.rb);
        }
    }
    return expect;
}

// ---------------------------------------------------------------------------
// HYBRID global-directory form with generalized slots (table.hpp): each slot
// keys on one field (1-D) or on the top bits of two fields (2-D grid), and
// every rule goes to the slot where it costs the fewest expected candidates.
// Rules whose best single field is wide (short prefixes on both addresses,
// wide port ranges) dominate the candidate lists of 1-D slots — for C5 the
// 4 % of rules whose best field covers >= 2^-12 of its key space account for
// ~5.7 of ~6.2 candidates per packet even with unbounded directories — and a
// 2-D key is selective for exactly those.
// ---------------------------------------------------------------------------

uint32_t ceil_log2(uint64_t x) {
    uint32_t b = 0;
    while ((uint64_t(1) << b) < x) ++b;
    return b;
}

uint32_t field_bits(uint32_t f) { return f < 2 ? 32u : 16u; }

uint32_t field_kind(uint32_t f, bool v6) {
    static const uint32_t k4[4] = {kKeyDst4, kKeySrc4, kKeyDport, kKeySport};
    static const uint32_t k6[4] = {kKeyDst6, kKeySrc6, kKeyDport, kKeySport};
    return f >= kFZero ? kKeyNone : (v6 ? k6[f] : k4[f]);
}

struct GSlot {
    uint32_t f1 = kFDst, b1 = 1, f2 = kFZero, b2 = 0;  // fields (SlotField) and radix bits
    std::vector<uint32_t> rules;                       // ascending rule order
    std::vector<uint32_t> dir, ents;
    uint32_t max_list = 0;
    uint64_t n_buckets() const { return uint64_t(1) << (b1 + b2); }
    // bucket index ranges [l1, h1] x [l2, h2] a rule with field ranges kr covers
    void span(const std::array<KeyRange, 4> &kr, uint64_t &l1, uint64_t &h1, uint64_t &l2, uint64_t &h2) const {
        const uint32_t s1 = field_bits(f1) - b1;
        l1 = kr[f1].lo >> s1;
        h1 = kr[f1].hi >> s1;
        l2 = h2 = 0;
        if (f2 < kFZero) {
            const uint32_t s2 = field_bits(f2) - b2;
            l2 = kr[f2].lo >> s2;
            h2 = kr[f2].hi >> s2;
        }
    }
    uint64_t count(const std::array<KeyRange, 4> &kr) const {
        uint64_t l1, h1, l2, h2;
        span(kr, l1, h1, l2, h2);
        return (h1 - l1 + 1) * (h2 - l2 + 1);
    }
    // bucket lists, ascending rule order within each
    void fill(const std::vector<std::array<KeyRange, 4>> &rr) {
        const size_t nb = n_buckets();
        std::vector<uint32_t> len(nb, 0);
        auto each = [&](uint32_t r, auto &&fn) {
            uint64_t l1, h1, l2, h2;
            span(rr[r], l1, h1, l2, h2);
            for (uint64_t t1 = l1; t1 <= h1; ++t1)
                for (uint64_t t2 = l2; t2 <= h2; ++t2) fn((t1 << b2) | t2);
        };
        for (uint32_t r : rules) each(r, [&](uint64_t t) { ++len[t]; });
        dir.assign(nb + 1, 0);
        max_list = 0;
        for (size_t t = 0; t < nb; ++t) {
            dir[t + 1] = dir[t] + len[t];
            max_list = std::max(max_list, len[t]);
        }
        ents.assign(dir[nb], 0);
        std::vector<uint32_t> at(dir.begin(), dir.end() - 1);
        for (uint32_t r : rules) each(r, [&](uint64_t t) { ents[at[t]++] = r; });
    }
};

// Candidates for a family of n rules: 1-D slots on every field, and (when
// `two_d` and the family is large) 2-D grids of the address pair and of an
// address with a port.  Radix widths: ~2 buckets per rule for the addresses
// (shrunk per slot once its rules are known).
std::vector<GSlot> slot_candidates(uint32_t n, bool two_d) {
    const uint32_t ba = std::min(17u, std::max(6u, ceil_log2(std::max<uint32_t>(n, 1)) + 1));
    const uint32_t bp = std::min(16u, ba - 2);
    std::vector<GSlot> c;
    auto add = [&](uint32_t f1, uint32_t b1, uint32_t f2, uint32_t b2) {
        GSlot g;
        g.f1 = f1, g.b1 = b1, g.f2 = f2, g.b2 = b2;
        c.push_back(g);
    };
    add(kFDst, ba, kFZero, 0);
    add(kFSrc, ba, kFZero, 0);
    add(kFDport, bp, kFZero, 0);
    add(kFSport, bp, kFZero, 0);
    if (two_d && n >= 1024) {
        const uint32_t a = std::min(9u, std::max(4u, ba / 2));
        add(kFDst, a, kFSrc, a);
        add(kFDst, a + 1, kFDport, 6);
        add(kFSrc, a + 1, kFDport, 6);
        add(kFDst, a + 1, kFSport, 6);
        add(kFSrc, a + 1, kFSport, 6);
    }
    return c;
}

// Expected candidates per packet above which a rule is scanned
// wave-uniformly (the residual list) instead of being listed: one uniform
// test per 64 packets beats ~64 * cost per-lane candidates past about this.
constexpr double kResidCost = 0.2;

// Assign rules (field ranges rr) to the slots: argmin over slots of
// span / buckets (expected candidates for a uniform packet) + mu * span
// (memory), mu the smallest keeping the lists within `budget` entries.
// choice[r] = slot index or -1 (residual).
void assign_g(const std::vector<std::array<KeyRange, 4>> &rr, const std::vector<GSlot> &slots, uint64_t budget,
              std::vector<int> &choice) {
    const size_t n = rr.size(), S = slots.size();
    std::vector<double> span(n * S), cost(n * S);
    for (size_t r = 0; r < n; ++r)
        for (size_t s = 0; s < S; ++s) {
            span[r * S + s] = double(slots[s].count(rr[r]));
            cost[r * S + s] = span[r * S + s] / double(slots[s].n_buckets());
        }
    auto run = [&](double mu) {
        uint64_t mem = 0;
        for (size_t r = 0; r < n; ++r) {
            int best = -1;
            double bv = 0, bc = 1e300;
            for (size_t s = 0; s < S; ++s) {
                const double v = cost[r * S + s] + mu * span[r * S + s];
                if (best < 0 || v < bv) { best = int(s); bv = v; }
                bc = std::min(bc, cost[r * S + s]);
            }
            if (bc >= kResidCost) best = -1;
            choice[r] = best;
            if (best >= 0) mem += uint64_t(span[r * S + best]);
        }
        return mem;
    };
    choice.assign(n, -1);
    if (run(0.0) <= budget) return;
    double lo = 0, hi = 1e-9;
    while (run(hi) > budget && hi < 1.0) hi *= 4;
    for (int it = 0; it < 40; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (run(mid) > budget) lo = mid; else hi = mid;
    }
    run(hi);
}

// Slots of one family: assign, drop empty slots (at most kMaxSlots kept: the
// least used is dropped and the rules re-assigned until they fit), then
// narrow each slot's radix to ~4 buckets per rule.
// Rules of each slot (and the residual list) from `choice`; empty slots dropped.
void distribute(const std::vector<int> &choice, std::vector<GSlot> &slots, std::vector<uint32_t> &resid) {
    resid.clear();
    for (auto &g : slots) g.rules.clear();
    for (uint32_t r = 0; r < choice.size(); ++r)
        if (choice[r] >= 0) slots[choice[r]].rules.push_back(r);
        else resid.push_back(r);
    slots.erase(std::remove_if(slots.begin(), slots.end(), [](const GSlot &g) { return g.rules.empty(); }),
                slots.end());
}

void plan_g(const std::vector<uint32_t> &recs, uint32_t rw, bool v6, uint32_t n, bool two_d, double slot_cost,
            bool global_dirs, std::vector<GSlot> &slots, std::vector<uint32_t> &resid,
            std::vector<std::array<KeyRange, 4>> &rr) {
    rr.assign(n, {});
    for (uint32_t r = 0; r < n; ++r) {
        KeyRange kr[4];
        rec_ranges(recs.data() + size_t(r) * rw, v6, kr);
        for (int k = 0; k < 4; ++k) rr[r][k] = kr[k];
    }
    slots = slot_candidates(n, two_d);
    const uint64_t budget = 4ull * n + 65536ull;
    std::vector<int> choice;
    while (true) {
        assign_g(rr, slots, budget, choice);
        std::vector<size_t> cnt(slots.size(), 0);
        for (int c : choice)
            if (c >= 0) ++cnt[c];
        std::vector<GSlot> kept;
        std::vector<size_t> kept_cnt;
        std::vector<int> remap(slots.size(), -1);
        for (size_t s = 0; s < slots.size(); ++s)
            if (cnt[s]) {
                remap[s] = int(kept.size());
                kept.push_back(slots[s]);
                kept_cnt.push_back(cnt[s]);
            }
        if (kept.size() <= kMaxSlots) {
            for (int &c : choice) c = c >= 0 ? remap[c] : -1;
            slots.swap(kept);
            break;
        }
        // too many slots in use: drop the least used one and re-assign
        const size_t worst = size_t(std::min_element(kept_cnt.begin(), kept_cnt.end()) - kept_cnt.begin());
        kept.erase(kept.begin() + long(worst));
        slots.swap(kept);
    }
    // A slot costs every packet of the family a directory read and a list
    // head: drop (cheapest first) slots whose rules would cost fewer than
    // `slot_cost` extra expected candidates per packet in their next-best slot.
    while (slot_cost > 0 && slots.size() > 1) {
        const size_t S = slots.size();
        std::vector<double> delta(S, 0.0);
        for (uint32_t r = 0; r < n; ++r) {
            const int c = choice[r];
            if (c < 0) continue;
            const double own = double(slots[c].count(rr[r])) / double(slots[c].n_buckets());
            double next = kResidCost;  // or the residual scan
            for (size_t s = 0; s < S; ++s)
                if (int(s) != c) next = std::min(next, double(slots[s].count(rr[r])) / double(slots[s].n_buckets()));
            delta[c] += std::max(0.0, next - own);
        }
        const size_t worst = size_t(std::min_element(delta.begin(), delta.end()) - delta.begin());
        if (delta[worst] >= slot_cost) break;
        slots.erase(slots.begin() + long(worst));
        assign_g(rr, slots, budget, choice);
    }
    distribute(choice, slots, resid);
    if (!global_dirs) return;  // LDS directories: fit_lds() sizes, re-assigns and fills
    for (auto &g : slots) {
        const uint32_t want = std::max(4u, ceil_log2(4ull * g.rules.size()));
        while (g.b1 + g.b2 > want) {
            if (g.f2 < kFZero && g.b2 > 1 && (g.b2 >= g.b1 || g.b1 <= 1)) --g.b2;
            else if (g.b1 > 1) --g.b1;
            else break;
        }
        g.fill(rr);
    }
}

// Bytes of a directory of nb buckets: plain u32, or two-level (table.hpp:
// a u32 base per 64 buckets + a u16 offset per bucket).
size_t gdir_bytes(uint64_t nb, bool dir16) {
    return dir16 ? 2 * (nb + 4) + 4 * ((nb >> kDir16GroupShift) + 2) : 4 * (nb + 1);
}

// Expected candidates per uniform packet of slot g at radix bits (b1, b2).
double gexpect(const GSlot &g, const std::vector<std::array<KeyRange, 4>> &rr, uint32_t b1, uint32_t b2) {
    GSlot t;
    t.f1 = g.f1, t.b1 = b1, t.f2 = g.f2, t.b2 = b2;
    double sum = 0;
    for (uint32_t r : g.rules) sum += double(t.count(rr[r]));
    return sum / double(t.n_buckets());
}

// LDS directories: narrow radix bits, one at a time, where a byte saved costs
// the fewest expected candidates (family-weighted), until both families'
// directories fit `budget`; then re-assign the rules to the final slots and
// build the lists.
void fit_lds(std::vector<GSlot> (&slots)[2], std::vector<uint32_t> (&resid)[2],
             const std::vector<std::array<KeyRange, 4>> (&rr)[2], const double (&weight)[2], size_t budget,
             bool dir16) {
    auto total = [&] {
        size_t b = 8;  // the empty directory
        for (int f = 0; f < 2; ++f)
            for (const auto &g : slots[f]) b += gdir_bytes(g.n_buckets(), dir16);
        return b;
    };
    std::vector<double> cur[2];
    for (int f = 0; f < 2; ++f)
        for (const auto &g : slots[f]) cur[f].push_back(gexpect(g, rr[f], g.b1, g.b2));
    while (total() > budget) {
        int bf = -1, bs = -1, bd = 0;
        double bscore = 0, bval = 0;
        for (int f = 0; f < 2; ++f)
            for (size_t s = 0; s < slots[f].size(); ++s) {
                const GSlot &g = slots[f][s];
                for (int d = 1; d <= (g.f2 < kFZero ? 2 : 1); ++d) {
                    const uint32_t b1 = g.b1 - (d == 1), b2 = g.b2 - (d == 2);
                    if ((d == 1 && g.b1 <= 1) || (d == 2 && g.b2 <= 1)) continue;
                    const double e = gexpect(g, rr[f], b1, b2);
                    const double saved = double(gdir_bytes(g.n_buckets(), dir16)) -
                                         double(gdir_bytes(uint64_t(1) << (b1 + b2), dir16));
                    const double score = weight[f] * (e - cur[f][s]) / std::max(saved, 1.0);
                    if (bf < 0 || score < bscore) { bf = f; bs = int(s); bd = d; bscore = score; bval = e; }
                }
            }
        if (bf < 0) break;  // every slot at one bucket bit
        GSlot &g = slots[bf][bs];
        if (bd == 1) --g.b1; else --g.b2;
        cur[bf][bs] = bval;
    }
    for (int f = 0; f < 2; ++f) {
        if (slots[f].empty()) continue;
        const size_t n = rr[f].size();
        std::vector<int> choice;
        assign_g(rr[f], slots[f], 4ull * n + 65536ull, choice);  // the final radix widths
        distribute(choice, slots[f], resid[f]);
        for (auto &g : slots[f]) g.fill(rr[f]);
    }
}

// Two-level directories are possible iff no 64-bucket group spans 65536+ entries.
bool gdir16_ok(const std::vector<GSlot> (&slots)[2]) {
    for (int f = 0; f < 2; ++f)
        for (const auto &g : slots[f])
            for (size_t t = 0; t < g.dir.size(); ++t)
                if (g.dir[t] - g.dir[(t >> kDir16GroupShift) << kDir16GroupShift] > 0xFFFFu) return false;
    return true;
}

void build_hybrid_g(const std::vector<uint32_t> &rec4, uint32_t n4, const std::vector<uint32_t> &rec6, uint32_t n6,
                    const CompileOptions &opt, size_t lds_budget, CompiledTable &out) {
    std::vector<GSlot> slots[2];
    std::vector<uint32_t> resid[2];
    std::vector<std::array<KeyRange, 4>> rr[2];
    const std::vector<uint32_t> *recs[2] = {&rec4, &rec6};
    const uint32_t rw[2] = {kRec4Dwords, kRec6Dwords}, nn[2] = {n4, n6};
    const bool lds = lds_budget > 0;
    for (int f = 0; f < 2; ++f)
        plan_g(*recs[f], rw[f], f == 1, nn[f], opt.slots2d != 0, opt.slot_cost, !lds, slots[f], resid[f], rr[f]);
    bool dir16 = false;
    if (lds) {  // directories staged in LDS: two-level when possible
        const double tot = std::max(1.0, double(n4) + double(n6));
        const double weight[2] = {double(n4) / tot, double(n6) / tot};
        const std::vector<GSlot> s0[2] = {slots[0], slots[1]};
        dir16 = opt.dir16;
        fit_lds(slots, resid, rr, weight, lds_budget, dir16);
        if (dir16 && !gdir16_ok(slots)) {
            dir16 = false;
            slots[0] = s0[0];
            slots[1] = s0[1];
            fit_lds(slots, resid, rr, weight, lds_budget, false);
        }
    }
    std::vector<uint32_t> &blob = out.blob;
    FamilyIndex *fi[2] = {&out.idx4, &out.idx6};
    // an empty directory {0, 0} for the kernels' unused slots, then the
    // directories (values: family-relative entry numbers; two-level: in the
    // group bases)
    out.off_empty_dir = 0;
    blob.insert(blob.end(), {0u, 0u});
    uint32_t dir_words[2][kMaxSlots] = {};
    for (int f = 0; f < 2; ++f)
        for (size_t k = 0; k < slots[f].size(); ++k) {
            const GSlot &g = slots[f][k];
            DimInfo &di = fi[f]->dims[k];
            di.off_dir = static_cast<uint32_t>(blob.size());
            if (!dir16) {
                blob.insert(blob.end(), g.dir.begin(), g.dir.end());
                dir_words[f][k] = static_cast<uint32_t>(g.dir.size());
                continue;
            }
            const size_t nb = g.dir.size() - 1;
            const size_t groups = (nb >> kDir16GroupShift) + 2;  // base[g + 1] stays readable
            for (size_t q = 0; q < groups; ++q) blob.push_back(g.dir[std::min(q << kDir16GroupShift, nb)]);
            dir_words[f][k] = static_cast<uint32_t>(groups);
            di.off_dir16 = static_cast<uint32_t>(blob.size());
            auto rel = [&](size_t t) -> uint32_t {
                return t <= nb ? g.dir[t] - g.dir[(t >> kDir16GroupShift) << kDir16GroupShift] : 0u;
            };
            const size_t words = (nb + 2) / 2 + 1;  // dword (t >> 1) + 1 stays readable
            for (size_t w = 0; w < words; ++w) blob.push_back(rel(2 * w) | rel(2 * w + 1) << 16);
        }
    while (blob.size() % 4) blob.push_back(0);
    out.lds_dwords = lds ? static_cast<uint32_t>(blob.size()) : 0u;
    for (int f = 0; f < 2; ++f) {
        const bool v6 = f == 1;
        const uint32_t ew = v6 ? kHybEnt6Dwords : kHybEnt4Dwords;
        fi[f]->entry_dwords = ew;
        fi[f]->off_ent_base = static_cast<uint32_t>(blob.size());
        fi[f]->used_slots = static_cast<uint32_t>(slots[f].size());
        for (size_t k = 0; k < slots[f].size(); ++k) {
            const GSlot &g = slots[f][k];
            DimInfo &di = fi[f]->dims[k];
            di.kind = field_kind(g.f1, v6);
            di.shift = field_bits(g.f1) - g.b1;
            di.kind2 = field_kind(g.f2, v6);
            di.bits2 = g.f2 < kFZero ? g.b2 : 0u;
            di.shift2 = g.f2 < kFZero ? field_bits(g.f2) - g.b2 : 0u;
            di.n_buckets = static_cast<uint32_t>(g.n_buckets());
            di.n_rules = static_cast<uint32_t>(g.rules.size());
            di.n_ent = g.ents.size();
            di.max_list = g.max_list;
            di.off_ent = static_cast<uint32_t>(blob.size());
            const uint32_t first = (di.off_ent - fi[f]->off_ent_base) / ew;  // family-relative entry numbers
            for (uint32_t t = 0; t < dir_words[f][k]; ++t) blob[di.off_dir + t] += first;
            for (uint32_t r : g.ents) emit_hyb_entry(recs[f]->data() + size_t(r) * rw[f], v6, r, blob);
        }
        fi[f]->off_resid = static_cast<uint32_t>(blob.size());
        fi[f]->n_resid = static_cast<uint32_t>(resid[f].size());
        for (uint32_t r : resid[f]) emit_hyb_entry(recs[f]->data() + size_t(r) * rw[f], v6, r, blob);
        while (blob.size() % 4) blob.push_back(0);
    }
    out.slots_g = true;
    out.flat_rounds = 4;
    out.off_rec4 = static_cast<uint32_t>(blob.size());
    for (uint32_t r = 0; r < n4; ++r) emit_cold(rec4.data() + size_t(r) * kRec4Dwords, false, blob);
    out.off_rec6 = static_cast<uint32_t>(blob.size());
    for (uint32_t r = 0; r < n6; ++r) emit_cold(rec6.data() + size_t(r) * kRec6Dwords, true, blob);
}

void build_hybrid(const std::vector<uint32_t> &rec4, uint32_t n4, const std::vector<uint32_t> &rec6, uint32_t n6,
                  const CompileOptions &opt, CompiledTable &out) {
    FamilyPlan plan[2];
    assign_family(rec4, kRec4Dwords, false, n4, plan[0]);
    assign_family(rec6, kRec6Dwords, true, n6, plan[1]);
    DimBuild *all[8];
    for (int f = 0; f < 2; ++f)
        for (int k = 0; k < 4; ++k) all[4 * f + k] = &plan[f].dims[k];
    double weight[8];
    for (int i = 0; i < 8; ++i) weight[i] = double(i < 4 ? n4 : n6) / double(std::max<uint32_t>(1, n4 + n6));
    // Policy: the flat walk over directories staged in LDS (flat-LDS) — it
    // beat the per-lane walks on C3 (0.519 vs 0.531 ms) and the flat walk
    // over 1 MiB global directories on C5 (0.918 vs 1.027 ms): lists sized
    // for LDS directories replicate short prefixes across far fewer buckets
    // and stay nearly L2-resident (C5: 3.8 MB of entries instead of ~10 MB),
    // profiles/r1_flat_lds/.
    // Tuning overrides (CompileOptions; experiments, tests): dir_bytes sets
    // the directory budget, flat forces the form (0 lane: INDEXED's inline
    // entries walked per lane; 1 flat with global directories; 2 flat-LDS);
    // directory budgets past LDS size always give the global flat form.
    const size_t tuned = opt.dir_bytes;
    const int force = opt.flat;
    const bool want16 = opt.dir16;
    const bool want8 = opt.dir8 && want16;
    if (force == 1 && !tuned) {  // global directories: generalized (1-D / 2-D) slots
        build_hybrid_g(rec4, n4, rec6, n6, opt, 0, out);
        return;
    }
    if (force == 2 && opt.slots2d == 2) {  // LDS directories, generalized slots (experiment)
        build_hybrid_g(rec4, n4, rec6, n6, opt, tuned ? tuned : kHybFlat4DirBytes, out);
        return;
    }
    size_t budget = tuned ? tuned : (force == 1 ? kHybFlatDirBytes : kHybLaneDirBytes);
    const bool lds_dirs = force != 1 && budget <= kHybLdsDirMaxBytes;
    const bool flat = force != 0 || !lds_dirs;
    // LDS directories: two-level, u8 offsets when every group fits (else u16, else plain u32)
    int fmt = lds_dirs ? (want8 ? 8 : want16 ? 16 : 0) : 0;
    const double expect = size_and_fill(all, weight, budget, fmt);
    // flat-LDS with many candidates per packet: 4 rounds in flight, whose
    // larger scratch takes some of the directory budget
    if (flat && lds_dirs && !tuned && expect > kHybFlat4Candidates) {
        budget = kHybFlat4DirBytes;
        size_and_fill(all, weight, budget, fmt);
        out.flat_uncond = 1;
    }
    // 4 rounds of candidate loads in flight for tables with many candidates
    // per packet, else 2: with the last window's rounds adaptive, C3 (1.45
    // candidates) runs 0.469 vs 0.473 ms at 2 (profiles/r2_valu/pfab/; round 1
    // measured 4 faster, 0.507 vs 0.540, before adaptive rounds)
    if (flat && lds_dirs) out.flat_rounds = expect > kHybFlat4Candidates ? 4 : 2;
    if (flat && lds_dirs && opt.uncond >= 0) out.flat_uncond = static_cast<uint32_t>(opt.uncond);
    // Fine 2-D slots (flat-LDS, positional slots 4..7: dst x dport, src x
    // dport, dst x sport, src x sport): a rule whose best single field is
    // wide — a short address prefix with the other address ANY, C5's
    // dominant candidates (1.5 per packet from /8 rules alone) — is
    // selective in an address-port pair.  Such a rule moves when the pair
    // grid's bucket covers a fraction of the key space below CompileOptions::fine_gain
    // of what its 1-D slot's bucket covers; the grids have fixed shapes (a
    // address bits x p port bits) and their directories come off the budget.
    DimBuild fine[2][4];
    bool any_fine = false;
    // does a directory's every group fit the offsets of form f (8: u8, 16: u16, 0: plain)?
    auto dir_fits = [](const std::vector<uint32_t> &dir, int f) {
        if (f == 0) return true;
        if (f == 4) {  // 4-bit counts: every list <= 15 entries
            for (size_t t = 0; t + 1 < dir.size(); ++t)
                if (dir[t + 1] - dir[t] > 15u) return false;
            return true;
        }
        const uint32_t gs = f == 8 ? kDir8GroupShift : kDir16GroupShift;
        const uint32_t lim = f == 8 ? 0xFFu : 0xFFFFu;
        for (size_t t = 0; t < dir.size(); ++t)
            if (dir[t] - dir[(t >> gs) << gs] > lim) return false;
        return true;
    };
    // the fine grids' directory bytes in form f (their shapes are fixed: only the form changes)
    auto fine_bytes_in = [&](int f) {
        size_t b = 0;
        for (int q = 0; q < 2; ++q)
            for (int k = 0; k < 4; ++k)
                if (!fine[q][k].rules.empty()) b += size_t(dir_form_bytes(double(fine[q][k].dir.size() - 1), f)) + 16;
        return b;
    };
    // 4-bit-count directories (flat-LDS positional forms): 1.67x the buckets
    // of the u8 form per LDS byte, so budget-bound slots get finer radixes
    // (C5: the address slots' longer prefixes collide in fewer buckets) at
    // a few more VALU per lookup; taken when the expected candidates drop
    if (flat && lds_dirs && fmt == 8 && opt.dir4 && !opt.coarse) {
        const double e8 = size_and_fill(all, weight, budget, 8);
        const double e4 = size_and_fill(all, weight, budget, 4);
        bool ok = e4 < 0.97 * e8;
        for (int i = 0; ok && i < 8; ++i) ok = dir_fits(all[i]->dir, 4);
        if (ok) fmt = 4;
        else size_and_fill(all, weight, budget, fmt);
    }
    // the plan before any rule moved to a grid: restored if the directories
    // ever degrade to the plain form, where the grids would not fit the budget
    FamilyPlan plan_1d[2];
    if (flat && lds_dirs && !tuned && opt.fine_a > 0 && !opt.coarse) {
        plan_1d[0] = plan[0];
        plan_1d[1] = plan[1];
        const uint32_t fa = static_cast<uint32_t>(opt.fine_a), fp = static_cast<uint32_t>(opt.fine_p);
        static const uint32_t f1s[4] = {kFDst, kFSrc, kFDst, kFSrc}, f2s[4] = {kFDport, kFDport, kFSport, kFSport};
        const uint32_t allowed = static_cast<uint32_t>(opt.fine_slots);  // bit k: positional slot 4 + k
        size_t fine_bytes = 0;
        for (int f = 0; f < 2; ++f) {
            FamilyPlan &pl = plan[f];
            const uint32_t n = f ? n6 : n4;
            if (n < kFineMinRules) continue;
            GSlot g[4];
            for (int k = 0; k < 4; ++k) g[k].f1 = f1s[k], g[k].b1 = fa, g[k].f2 = f2s[k], g[k].b2 = fp;
            std::vector<std::vector<uint32_t>> moved(4);
            std::vector<char> gone(n, 0);
            for (int d = 0; d < 4; ++d) {
                const DimBuild &db = pl.dims[d];
                for (size_t i = 0; i < db.rules.size(); ++i) {
                    const uint32_t r = db.rules[i];
                    const double own = double((db.ranges[i].hi >> db.shift) - (db.ranges[i].lo >> db.shift) + 1) /
                                       double(uint64_t(1) << db.rb);
                    int best = -1;
                    double bc = own * opt.fine_gain;
                    for (int k = 0; k < 4; ++k) {
                        if (!((allowed >> k) & 1u)) continue;
                        const double c = double(g[k].count(pl.rr[r])) / double(g[k].n_buckets());
                        if (c < bc) { bc = c; best = k; }
                    }
                    if (best >= 0) { moved[best].push_back(r); gone[r] = 1; }
                }
            }
            for (int k = 0; k < 4; ++k) {
                if (moved[k].size() < size_t(opt.fine_min)) continue;  // not worth a slot: the rules stay
                std::sort(moved[k].begin(), moved[k].end());
                g[k].rules = moved[k];
                g[k].fill(pl.rr);
                // A grid whose lists overflow the current form's offsets
                // sheds the rules that touch an overflowing group of buckets
                // (they stay in their 1-D slots): in the wider form its
                // directory would outgrow the bytes taken off the budget.
                // Left with fewer than fine_min rules, it is not built.
                for (int it = 0; it < 8 && !dir_fits(g[k].dir, fmt); ++it) {
                    // (4-bit counts: the overflowing buckets themselves, gs 0)
                    const uint32_t gs = fmt == 4 ? 0u : fmt == 8 ? kDir8GroupShift : kDir16GroupShift;
                    const uint32_t lim = fmt == 8 ? 0xFFu : 0xFFFFu;
                    const std::vector<uint32_t> &dir = g[k].dir;
                    std::vector<char> hot((dir.size() >> gs) + 1, 0);
                    for (size_t t = 0; t < dir.size(); ++t) {
                        if (fmt == 4) {
                            if (t + 1 < dir.size() && dir[t + 1] - dir[t] > 15u) hot[t] = 1;
                        } else if (dir[t] - dir[(t >> gs) << gs] > lim) {
                            hot[t >> gs] = 1;
                        }
                    }
                    std::vector<uint32_t> keep;
                    for (uint32_t r : g[k].rules) {
                        uint64_t l1, h1, l2, h2;
                        g[k].span(pl.rr[r], l1, h1, l2, h2);
                        bool touch = false;
                        for (uint64_t t1 = l1; t1 <= h1 && !touch; ++t1)
                            for (uint64_t t2 = l2; t2 <= h2 && !touch; ++t2)
                                touch = hot[((t1 << g[k].b2) | t2) >> gs] != 0;
                        if (!touch) keep.push_back(r);
                    }
                    g[k].rules.swap(keep);
                    g[k].fill(pl.rr);
                }
                if (!dir_fits(g[k].dir, fmt) || g[k].rules.size() < size_t(opt.fine_min)) {
                    g[k].rules.clear();
                    continue;
                }
                DimBuild &fd = fine[f][k];
                fd.kind = field_kind(g[k].f1, f == 1);
                fd.key_bits = 32;
                fd.rb = g[k].b1 + g[k].b2;
                fd.shift = 32 - g[k].b1;
                fd.kind2 = field_kind(g[k].f2, f == 1);
                fd.bits2 = g[k].b2;
                fd.shift2 = 16 - g[k].b2;
                fd.rules = g[k].rules;
                fd.dir = g[k].dir;
                fd.ents = g[k].ents;
                fd.max_list = g[k].max_list;
                fine_bytes += size_t(dir_form_bytes(double(g[k].n_buckets()), fmt)) + 16;
                any_fine = true;
            }
            // Coarse address grids (slots 6 / 7 when no fine grid uses them):
            // a dst / src rule whose prefix spans >= 2^cgrid buckets of its
            // 1-D slot is replicated that many times; in a grid on the same
            // address with radix rb - cgrid (no port bits) it is a candidate
            // for exactly the same packets with 2^cgrid times fewer copies.
            for (int c = 0; opt.cgrid > 0 && c < 2; ++c) {
                // the first positional grid slot (4..7) on this address that no fine grid takes
                const uint32_t field = c == 0 ? kFDst : kFSrc;
                int k = -1;
                for (int q = 0; q < 4 && k < 0; ++q)
                    if (f1s[q] == field && !((allowed >> q) & 1u) && fine[f][q].rules.empty()) k = q;
                if (k < 0) continue;
                const DimBuild &db = pl.dims[c];
                if (db.rb < uint32_t(opt.cgrid) + 6u) continue;
                const uint32_t wide = 1u << opt.cgrid;
                std::vector<uint32_t> mv;
                for (size_t i = 0; i < db.rules.size(); ++i) {
                    const uint32_t r = db.rules[i];
                    if (!gone[r] && (db.ranges[i].hi >> db.shift) - (db.ranges[i].lo >> db.shift) + 1 >= wide)
                        mv.push_back(r);
                }
                if (mv.size() < size_t(opt.fine_min)) continue;
                std::sort(mv.begin(), mv.end());
                GSlot gc;
                gc.f1 = field;
                gc.b1 = db.rb - uint32_t(opt.cgrid);
                gc.f2 = f2s[k];  // (no port bits: b2 = 0)
                gc.b2 = 0;
                gc.rules = mv;
                gc.fill(pl.rr);
                if (!dir_fits(gc.dir, fmt)) continue;
                for (uint32_t r : mv) gone[r] = 1;
                DimBuild &fd = fine[f][k];
                fd.kind = field_kind(gc.f1, f == 1);
                fd.key_bits = 32;
                fd.rb = gc.b1;
                fd.shift = 32 - gc.b1;
                fd.kind2 = field_kind(gc.f2, f == 1);
                fd.bits2 = 0;
                fd.shift2 = 16;
                fd.rules = gc.rules;
                fd.dir = gc.dir;
                fd.ents = gc.ents;
                fd.max_list = gc.max_list;
                fine_bytes += size_t(dir_form_bytes(double(gc.n_buckets()), fmt)) + 16;
                any_fine = true;
            }
            for (int d = 0; d < 4; ++d) {  // the moved rules leave their 1-D slots
                DimBuild &db = pl.dims[d];
                std::vector<uint32_t> keep;
                std::vector<KeyRange> keep_r;
                for (size_t i = 0; i < db.rules.size(); ++i) {
                    const uint32_t r = db.rules[i];
                    bool left = false;
                    if (gone[r])
                        for (int k = 0; k < 4 && !left; ++k)
                            left = !fine[f][k].rules.empty() && std::binary_search(fine[f][k].rules.begin(),
                                                                                   fine[f][k].rules.end(), r);
                    if (!left) {
                        keep.push_back(r);
                        keep_r.push_back(db.ranges[i]);
                    }
                }
                db.rules.swap(keep);
                db.ranges.swap(keep_r);
            }
        }
        if (any_fine) size_and_fill(all, weight, budget > fine_bytes ? budget - fine_bytes : 1024, fmt);
    }
    // Coarse address slots (flat-LDS): a rule whose prefix is shorter than
    // its address slot's radix is replicated into 2^(radix - length) buckets
    // (C5 at 15-bit radixes: 3.1-3.5 entries per rule, 6.4 MB of entries,
    // L2 hit rate 0.55).  Rules at least kCoarseGap bits shorter than the
    // radix move to a second slot on the same field whose radix is capped at
    // that threshold: the same candidates per packet (a bucket no finer than
    // the prefix), far fewer copies.  The slots are then compacted per family
    // (generalized slots: each keyed on its field, CompiledTable::slots_g).
    // Measured slower on C5 (table 7.7 -> 3.7 MB, L2 traffic down, but the
    // two extra slots' lookups and marks cost more: 0.722 vs 0.649 ms), so
    // it is a tuning option (NFFACL_TUNE_COARSE=1), off by default.
    DimBuild coarse[2][2];
    std::vector<DimBuild *> ext(all, all + 8);
    std::vector<double> wext(weight, weight + 8);
    bool compact = false;
    if (flat && lds_dirs && opt.coarse) {
        for (int f = 0; f < 2; ++f)
            for (int k = 0; k < 2; ++k) {  // dst, src
                DimBuild &d = plan[f].dims[k];
                if (d.rules.size() < kCoarseMinRules || d.rb < kCoarseGap + 8) continue;
                const uint32_t thr = d.rb - kCoarseGap;
                DimBuild &c = coarse[f][k];
                c.kind = d.kind;
                c.key_bits = d.key_bits;
                c.max_rb = thr;
                const uint64_t wide = uint64_t(1) << (d.key_bits - thr);  // prefix shorter than thr bits
                std::vector<uint32_t> keep;
                std::vector<KeyRange> keep_r;
                for (size_t i = 0; i < d.rules.size(); ++i) {
                    const bool move = uint64_t(d.ranges[i].hi) - d.ranges[i].lo + 1 > wide;
                    (move ? c.rules : keep).push_back(d.rules[i]);
                    (move ? c.ranges : keep_r).push_back(d.ranges[i]);
                }
                if (c.rules.size() < kCoarseMinMoved) {  // not worth a slot: keep them
                    c.rules.clear();
                    c.ranges.clear();
                    continue;
                }
                d.rules.swap(keep);
                d.ranges.swap(keep_r);
                ext.push_back(&c);
                wext.push_back(weight[4 * f]);
                compact = true;
            }
        if (compact) size_and_fill(ext.data(), wext.data(), budget, fmt, static_cast<int>(ext.size()));
    }
    const int nd = static_cast<int>(ext.size());
    // a group whose lists overflow its offsets: the next wider form, re-sized for the same budget
    auto form_fits = [&](int f) {
        for (int i = 0; i < nd; ++i)
            if (!dir_fits(ext[i]->dir, f)) return false;
        return true;
    };
    auto fine_fits = [&](int f) {
        for (int q = 0; q < 2; ++q)
            for (int k = 0; k < 4; ++k)
                if (!dir_fits(fine[q][k].dir, f)) return false;
        return true;
    };
    while (!form_fits(fmt) || !fine_fits(fmt)) {
        fmt = fmt == 4 ? 8 : fmt == 8 && want16 ? 16 : 0;
        if (any_fine && fmt == 0) {  // plain directories: no room for the grids, their rules go back
            plan[0] = plan_1d[0];
            plan[1] = plan_1d[1];
            for (auto &ff : fine)
                for (DimBuild &fd : ff) fd = DimBuild{};
            any_fine = false;
        }
        // the 1-D slots re-sized for what the grids leave of the budget in the new form
        const size_t fb = any_fine ? fine_bytes_in(fmt) : 0;
        size_and_fill(ext.data(), wext.data(), budget > fb ? budget - fb : 1024, fmt, nd);
    }
    const bool dir16 = fmt != 0;
    out.dir8 = fmt == 8 ? 1u : fmt == 4 ? 2u : 0u;
    // slot order per family: positional [dst, src, dport, sport] (empty ones
    // included), or compacted (non-empty slots only, coarse ones last)
    std::vector<DimBuild *> order[2];
    for (int f = 0; f < 2; ++f) {
        for (int k = 0; k < 4; ++k)
            if (!compact || !plan[f].dims[k].rules.empty()) order[f].push_back(&plan[f].dims[k]);
        for (int k = 0; k < 2; ++k)
            if (compact && !coarse[f][k].rules.empty()) order[f].push_back(&coarse[f][k]);
        if (any_fine)  // positional 4..7 (an empty slot: an empty directory of two buckets)
            for (int k = 0; k < 4; ++k) {
                DimBuild &fd = fine[f][k];
                if (fd.rules.empty()) {
                    fd.kind = field_kind(k & 1 ? kFSrc : kFDst, f == 1);
                    fd.kind2 = field_kind(k < 2 ? kFDport : kFSport, f == 1);
                    fd.rb = 1;
                    fd.shift = 31;
                    fd.bits2 = 0;
                    fd.shift2 = 16;
                    fd.dir.assign(3, 0);
                    fd.ents.clear();
                    fd.max_list = 0;
                }
                order[f].push_back(&fd);
            }
    }
    std::vector<uint32_t> &blob = out.blob;
    FamilyIndex *fi[2] = {&out.idx4, &out.idx6};
    const std::vector<uint32_t> *recs[2] = {&rec4, &rec6};
    const uint32_t rw[2] = {kRec4Dwords, kRec6Dwords};
    if (compact) {  // an empty directory {0, 0} for the kernels' unused slots (staged with the rest)
        out.off_empty_dir = 0;
        blob.insert(blob.end(), {0u, 0u});
    }
    // the directories first: the LDS image of the lane and flat-LDS forms
    uint32_t dir_words[2][kMaxSlots];  // directory words holding entry numbers (base words when two-level)
    for (int f = 0; f < 2; ++f)
        for (size_t k = 0; k < order[f].size(); ++k) {
            const std::vector<uint32_t> &dir = order[f][k]->dir;
            DimInfo &di = fi[f]->dims[k];
            di.off_dir = static_cast<uint32_t>(blob.size());
            if (!dir16) {
                blob.insert(blob.end(), dir.begin(), dir.end());
                dir_words[f][k] = static_cast<uint32_t>(dir.size());
                continue;
            }
            const size_t nb = dir.size() - 1;
            const uint32_t gs = out.dir8 == 2 ? kDir4GroupShift : out.dir8 ? kDir8GroupShift : kDir16GroupShift;
            const size_t groups = (nb >> gs) + 2;  // base[g + 1] stays readable
            for (size_t g = 0; g < groups; ++g) blob.push_back(dir[std::min(g << gs, nb)]);
            dir_words[f][k] = static_cast<uint32_t>(groups);
            if (out.dir8 == 2 && blob.size() % 2) blob.push_back(0);  // counts: 8-byte aligned dword pairs
            di.off_dir16 = static_cast<uint32_t>(blob.size());
            di.dir8 = out.dir8;
            if (out.dir8 == 2) {  // 4-bit counts, 8 per dword; group g = dwords 2g, 2g + 1
                const size_t words = 2 * ((nb >> kDir4GroupShift) + 2);
                for (size_t w = 0; w < words; ++w) {
                    uint32_t x = 0;
                    for (size_t i = 0; i < 8; ++i) {
                        const size_t t = 8 * w + i;
                        if (t < nb) x |= (dir[t + 1] - dir[t]) << (4 * i);
                    }
                    blob.push_back(x);
                }
                continue;
            }
            auto rel = [&](size_t t) -> uint32_t { return t <= nb ? dir[t] - dir[(t >> gs) << gs] : 0u; };
            if (out.dir8) {
                const size_t words = (nb + 4) / 4 + 1;  // dword (t >> 2) + 1 stays readable
                for (size_t w = 0; w < words; ++w)
                    blob.push_back(rel(4 * w) | rel(4 * w + 1) << 8 | rel(4 * w + 2) << 16 | rel(4 * w + 3) << 24);
                continue;
            }
            const size_t words = (nb + 2) / 2 + 1;  // dword (t >> 1) + 1 stays readable
            for (size_t w = 0; w < words; ++w) blob.push_back(rel(2 * w) | rel(2 * w + 1) << 16);
        }
    while (blob.size() % 4) blob.push_back(0);
    // flat-LDS positional forms: the slot parameter block (table.hpp
    // kFlatParamDwords), staged with the directories (offsets < 2^16 dwords)
    if (flat && lds_dirs && !compact) {  // (the image is < 2^16 dwords: kHybLdsDirMaxBytes)
        out.off_params = static_cast<uint32_t>(blob.size());
        for (uint32_t k = 0; k < kMaxSlots; ++k) {
            uint32_t w[kFlatParamDwords] = {0, 0, 0, 0};
            for (int f = 0; f < 2; ++f) {
                const uint32_t sh = 16u * f;
                if (k >= order[f].size()) continue;
                const DimBuild &d = *order[f][k];
                const DimInfo &di = fi[f]->dims[k];
                w[0] |= (d.shift & 0xFFFFu) << sh;
                w[1] |= (di.off_dir & 0xFFFFu) << sh;
                w[2] |= (di.off_dir16 & 0xFFFFu) << sh;
                w[3] |= ((d.bits2 & 0xFFu) | (d.shift2 & 0xFFu) << 8) << sh;
            }
            blob.insert(blob.end(), w, w + kFlatParamDwords);
        }
    }
    out.lds_dwords = lds_dirs ? static_cast<uint32_t>(blob.size()) : 0u;
    for (int f = 0; f < 2; ++f) {
        const bool v6 = f == 1;
        // lane form: INDEXED's inline entries (exact, output inline — a hit
        // costs no further read); flat form: compact entries + cold records
        const uint32_t ew = flat ? (v6 ? kHybEnt6Dwords : kHybEnt4Dwords) : (v6 ? kEnt6Dwords : kEnt4Dwords);
        fi[f]->entry_dwords = ew;
        fi[f]->off_ent_base = static_cast<uint32_t>(blob.size());
        for (size_t k = 0; k < order[f].size(); ++k) {
            DimBuild &d = *order[f][k];
            DimInfo &di = fi[f]->dims[k];
            di.kind = d.kind;
            di.shift = d.shift;
            di.kind2 = d.kind2;
            di.shift2 = d.shift2;
            di.bits2 = d.bits2;
            di.n_buckets = 1u << d.rb;
            di.n_rules = static_cast<uint32_t>(d.rules.size());
            di.n_ent = d.ents.size();
            di.max_list = d.max_list;
            di.off_ent = static_cast<uint32_t>(blob.size());
            if (flat) {  // directory values: family-relative entry numbers
                const uint32_t first = (di.off_ent - fi[f]->off_ent_base) / ew;
                for (uint32_t t = 0; t < dir_words[f][k]; ++t) blob[di.off_dir + t] += first;
                for (uint32_t r : d.ents) emit_hyb_entry(recs[f]->data() + size_t(r) * rw[f], v6, r, blob);
            } else {     // relative to off_ent, as INDEXED
                for (uint32_t r : d.ents) emit_entry(recs[f]->data() + size_t(r) * rw[f], v6, r, blob);
                if (d.ents.empty()) blob.insert(blob.end(), ew, 0u);  // keep entry 0 addressable
            }
            if (!d.rules.empty()) fi[f]->used_slots = static_cast<uint32_t>(k + 1);
        }
        fi[f]->off_resid = static_cast<uint32_t>(blob.size());
        fi[f]->n_resid = static_cast<uint32_t>(plan[f].resid.size());
        for (uint32_t r : plan[f].resid) {
            if (flat) emit_hyb_entry(recs[f]->data() + size_t(r) * rw[f], v6, r, blob);
            else emit_entry(recs[f]->data() + size_t(r) * rw[f], v6, r, blob);
        }
        while (blob.size() % 4) blob.push_back(0);
    }
    out.slots_g = compact;
    if (flat) {
        out.off_rec4 = static_cast<uint32_t>(blob.size());
        for (uint32_t r = 0; r < n4; ++r) emit_cold(rec4.data() + size_t(r) * kRec4Dwords, false, blob);
        out.off_rec6 = static_cast<uint32_t>(blob.size());
        for (uint32_t r = 0; r < n6; ++r) emit_cold(rec6.data() + size_t(r) * kRec6Dwords, true, blob);
    }
}

// Indexed tables encode id_mask as one bit and the rule index in 23 bits.
bool indexable(const nffacl_rules &rules) {
    if (rules.ip4.size() >= kMaxIndexedRules || rules.ip6.size() >= kMaxIndexedRules) return false;
    for (const auto &r : rules.ip4)
        if (r.l4.id_mask != 0 && r.l4.id_mask != 0xFF) return false;
    for (const auto &r : rules.ip6)
        if (r.l4.id_mask != 0 && r.l4.id_mask != 0xFF) return false;
    return true;
}

}  // namespace

bool env_knob(const char *name, long lo, long hi, long &v, bool &set, std::string &err) {
    const char *s = std::getenv(name);
    set = s && *s;
    if (!set) return true;
    char *end = nullptr;
    v = std::strtol(s, &end, 10);
    if (*end != '\0' || v < lo || v > hi) {
        err = std::string(name) + "=" + s + ": expected an integer in [" + std::to_string(lo) + ", " +
              std::to_string(hi) + "]";
        return false;
    }
    return true;
}

bool CompileOptions::from_env(CompileOptions &o, std::string &err) {
    o = CompileOptions{};
    long v = 0;
    bool set = false;
    if (!env_knob("NFFACL_TUNE_FLAT", 0, 2, v, set, err)) return false;
    if (set) o.flat = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DIR_KB", 1, 1 << 20, v, set, err)) return false;
    if (set) o.dir_bytes = size_t(v) * 1024;
    if (!env_knob("NFFACL_TUNE_DIR16", 0, 1, v, set, err)) return false;
    if (set) o.dir16 = v != 0;
    if (!env_knob("NFFACL_TUNE_DIR4", 0, 1, v, set, err)) return false;
    if (set) o.dir4 = v != 0;
    if (!env_knob("NFFACL_TUNE_DIR8", 0, 1, v, set, err)) return false;
    if (set) o.dir8 = v != 0;
    if (!env_knob("NFFACL_TUNE_COARSE", 0, 1, v, set, err)) return false;
    if (set) o.coarse = v != 0;
    if (!env_knob("NFFACL_TUNE_UNCOND", 0, 1, v, set, err)) return false;
    if (set) o.uncond = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_SLOTS2D", 0, 2, v, set, err)) return false;
    if (set) o.slots2d = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_SLOT_COST", 0, 1000, v, set, err)) return false;
    if (set) o.slot_cost = double(v) / 100.0;
    if (!env_knob("NFFACL_TUNE_FINE_A", 0, 12, v, set, err)) return false;
    if (set) o.fine_a = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_FINE_P", 1, 8, v, set, err)) return false;
    if (set) o.fine_p = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_FINE_G", 1, 100, v, set, err)) return false;
    if (set) o.fine_gain = double(v) / 100.0;
    if (!env_knob("NFFACL_TUNE_FINE_MIN", 1, 1 << 20, v, set, err)) return false;
    if (set) o.fine_min = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_FINE_SLOTS", 0, 15, v, set, err)) return false;
    if (set) o.fine_slots = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DIR_PER_RULE", 1, 64, v, set, err)) return false;
    if (set) o.dir_per_rule = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_CGRID", 0, 12, v, set, err)) return false;
    if (set) o.cgrid = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DIR_SB", 0, 100, v, set, err)) return false;
    if (set) o.dir_sbias = static_cast<int>(v);
    return true;
}

bool compile_table(const nffacl_rules &rules, int algo, const CompileOptions &opt, CompiledTable &out,
                   std::string &err) {
    if (algo != NFFACL_ALGO_AUTO && algo != NFFACL_ALGO_LINEAR && algo != NFFACL_ALGO_INDEXED &&
        algo != NFFACL_ALGO_HYBRID) {
        err = "unknown algorithm";
        return false;
    }
    out = CompiledTable{};
    g_dir_per_rule = static_cast<size_t>(opt.dir_per_rule);
    g_dir_sbias = double(opt.dir_sbias) / 100.0;
    std::vector<uint32_t> rec4, rec6;
    rec4.reserve(rules.ip4.size() * kRec4Dwords);
    rec6.reserve(rules.ip6.size() * kRec6Dwords);
    for (const auto &r : rules.ip4)
        if (emit_rec4(r, rec4)) ++out.n4;
    for (const auto &r : rules.ip6)
        if (emit_rec6(r, rec6)) ++out.n6;
    // AUTO = INDEXED whenever encodable: with the lane-contiguous loads even
    // 5 rules classify faster indexed (C1: 70.2 vs 67.3 Gpps LINEAR,
    // profiles/r1_configs_k/) — unless its inline table outgrows LDS, where
    // HYBRID keeps the directories in LDS and the lists compact in HBM.
    if (algo == NFFACL_ALGO_HYBRID && !hybrid_encodable(rec4, out.n4, rec6, out.n6)) algo = NFFACL_ALGO_INDEXED;
    // HYBRID, and never a flat-LDS image past the staged-image limit (the
    // launch refuses one, table_consistent): should the fine 2-D grids push
    // it there (layout knobs: NFFACL_TUNE_FINE_A = 10 at C5 made 271 KB),
    // build without them, and failing that with global directories
    auto hybrid = [&](uint32_t n4, uint32_t n6) {
        auto build = [&](const CompileOptions &o) {
            out = CompiledTable{};
            out.n4 = n4;
            out.n6 = n6;
            out.algo = NFFACL_ALGO_HYBRID;
            build_hybrid(rec4, n4, rec6, n6, o, out);
        };
        auto over = [&] {  // (table_consistent's limits: flat-LDS image / lane-form directories)
            const size_t b = size_t(out.lds_dwords) * sizeof(uint32_t);
            return out.idx4.entry_dwords == kHybEnt4Dwords ? b > kHybLdsDirMaxBytes : b > kLdsTableBytes;
        };
        build(opt);
        if (!over()) return;
        CompileOptions o = opt;
        o.fine_a = 0;
        build(o);
        if (!over()) return;
        o.flat = 1;
        build(o);
    };
    if (algo == NFFACL_ALGO_HYBRID) {
        hybrid(out.n4, out.n6);
    } else if (algo != NFFACL_ALGO_LINEAR && indexable(rules)) {
        out.algo = NFFACL_ALGO_INDEXED;
        build_family(rec4, kRec4Dwords, false, out.n4, out.blob, out.idx4);
        build_family(rec6, kRec6Dwords, true, out.n6, out.blob, out.idx6);
        if (algo == NFFACL_ALGO_AUTO && out.blob.size() * 4 > kLdsTableBytes &&
            hybrid_encodable(rec4, out.n4, rec6, out.n6)) {
            hybrid(out.n4, out.n6);
        }
    } else {
        out.algo = NFFACL_ALGO_LINEAR;
        out.off_rec4 = 0;
        out.off_rec6 = static_cast<uint32_t>(rec4.size());
        out.blob = rec4;
        out.blob.insert(out.blob.end(), rec6.begin(), rec6.end());
    }
    if (out.blob.empty()) out.blob.push_back(0);  // keep a valid allocation
    while (out.blob.size() % 4) out.blob.push_back(0);
    bool any = true;
    for (size_t i = 4; i < rec4.size() && any; i += kRec4Dwords) any = (rec4[i] & kMetaPortCheck) == 0u;
    for (size_t i = 16; i < rec6.size() && any; i += kRec6Dwords) any = (rec6[i] & kMetaPortCheck) == 0u;
    out.ports_any = any ? 1u : 0u;
    return true;
}

}  // namespace nffacl
