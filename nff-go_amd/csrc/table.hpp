// table.hpp — device table formats shared by the host compiler (compile.cpp)
// and the HIP kernels (engine.hip).  Internal to libnffacl.
//
// Packet fields are taken straight from little-endian dwords of the slot
// (dword k = wire bytes 4k..4k+3).  Every field behind the Ethernet header sits
// at a wire offset = 2 (mod 4), so a field is one funnel
// shift of two neighbouring dwords, and the extracted IPv4 address is exactly
// the reference's types.IPv4Address (LE u32 of the wire bytes,
// packet/acl.go:400-402).  Rule words therefore compare against packet words
// without any byte swapping.
#pragma once

#include <cstdint>

namespace nffacl {

// ---- linear table: one record per rule, scanned in file order ------------
//
// IPv4 record, 8 dwords (32 B, one s_load_dwordx8):
//   [0] src_addr  [1] src_mask  [2] dst_addr  [3] dst_mask
//   [4] meta = id | id_mask << 8 | (port_check << 16)
//   [5] lo = src_port_min | dst_port_min << 16
//   [6] hi = src_port_max | dst_port_max << 16
//   [7] output_number
// IPv6 record, 20 dwords (80 B):
//   [0..3] src_addr  [4..7] src_mask  [8..11] dst_addr  [12..15] dst_mask
//   (each 16-byte field as 4 LE dwords of its wire bytes)
//   [16] meta  [17] lo  [18] hi  [19] output_number
constexpr uint32_t kRec4Dwords = 8;
constexpr uint32_t kRec6Dwords = 20;
constexpr uint32_t kMetaPortCheck = 1u << 16;

// ---- indexed table -------------------------------------------------------
//
// The rules of one family are split over four key "slots" (destination
// address, source address, destination port, source port).  Each rule is
// assigned to exactly one slot d — the one where its constraint is most
// selective — and filed in d's radix-bucket index: bucket t covers keys
// [t << shift, ((t+1) << shift) - 1] and lists, in ascending rule order, every
// rule of d whose key range meets the bucket, as an inline entry (the full
// rule, so a candidate costs one table read):
//   dir[t] .. dir[t+1]      (u32, 2^(keybits - shift) + 1 entries)
//   entries[...]            (kEnt4Dwords / kEnt6Dwords each)
// A packet's first match is the minimum over slots of the first listed rule
// (in rule order) that passes the full rule test, so a bucket only has to
// list a superset of the rules that can match a key in it — the projection of
// a non-prefix mask to its leading-ones run, or of an IPv6 address to its top
// 32 bits, keeps the result exact.  Rules without any selective key go to the
// family's residual entry list, scanned wave-uniformly in rule order.
//
// Entry (IPv4, 8 dwords = 2 x 16 B; IPv6 adds 12 extension dwords):
//   [0] src word  [1] src mask  [2] dst word  [3] dst mask     (IPv6: top 32 bits)
//   [4] meta = id | exact << 8 | rule_index << 9   (exact: id_mask == 0xff)
//   [5] lo = sport_min | dport_min << 16   [6] hi = sport_max | dport_max << 16
//   [7] output_number
//   IPv6 [8..19]: src[1..3], src_mask[1..3], dst[1..3], dst_mask[1..3]
// Indexed tables therefore need id_mask in {0, 0xff} (what the parsers
// produce) and < 2^23 rules per family; other rule sets compile LINEAR.
constexpr uint32_t kEnt4Dwords = 8;
constexpr uint32_t kEnt6Dwords = 20;
constexpr uint32_t kEntIndexShift = 9;
constexpr uint32_t kEntExact = 1u << 8;
constexpr uint32_t kMaxIndexedRules = 1u << 23;

// ---- hybrid table (tables whose inline index outgrows LDS) ---------------
//
// Same slot assignment and ascending bucket lists as the indexed table, with
// the eight directories (both families) first in the blob, in one of three
// forms:
//  * flat-LDS (default; lds_dwords > 0, entry_dwords == kHybEnt4Dwords): the
//    directories, radix widths chosen to fit kHybLaneDirBytes, are the LDS
//    image — two-level (kDir16GroupShift) when every group fits u16
//    offsets — holding family-relative entry numbers (two-level: in the base
//    words); a wave tests its packets' candidates 64 at a time, list entries
//    exact (below);
//  * lane form (forced; lds_dwords > 0, INDEXED entry sizes): the same LDS
//    directories, values relative to the slot's entries; the lists hold
//    INDEXED's inline entries read from global memory, each lane walking its
//    own lists;
//  * flat form (forced, or directory budgets past LDS; lds_dwords == 0):
//    plain u32 directories read from global memory, values and entries as
//    flat-LDS; with generalized slots (CompiledTable::slots_g) each slot keys
//    on one field or on a 2-D grid of two fields' top bits.
// A flat-form list entry is EXACT — a candidate needs no second read:
//   IPv4, 6 dwords (24 B):
//      [0] src word, big-endian value   [1] dst word, big-endian value
//      [2] meta = id | exact << 8 | rule_index << 9          (as inline)
//      [3] lo = sport_min | dport_min << 16   [4] hi = sport_max | dport_max << 16
//          (IPv4 rules without a port check: 0 / 0xffffffff)
//      [5] src_len | dst_len << 8 | out << 16
//   IPv6, 12 dwords (48 B): the same six words with the top 32 address bits
//      and prefix lengths 0..128, then [6..8] src words 1..3, [9..11] dst
//      words 1..3 (big-endian values).
// `out` is the OutputNumber when < kHybOutEscape; otherwise it is read from
// the family's output array (one u32 per rule, in rule order; off_rec4 /
// off_rec6).  Loads are 12-byte (dwordx3): two per IPv4 entry, four per IPv6.
// The hybrid forms encode only CIDR masks and id_mask in {0, 0xff} (what
// the parsers produce); other rule sets compile INDEXED.
constexpr uint32_t kHybEnt4Dwords = 6;
constexpr uint32_t kHybEnt6Dwords = 12;
constexpr uint32_t kHybOutShift = 16;
constexpr uint32_t kHybOutEscape = 0xFFFFu;  // output number >= this: read from the output array
// Directory budgets (both families), see above.  128 KiB of LDS directories
// leave one 1024-thread workgroup per CU; measured faster than 64 KiB with
// two (C3: 0.64 vs 0.69 ms, profiles/r1_hybrid/).
constexpr size_t kHybLaneDirBytes = 128 * 1024;
constexpr size_t kHybFlatDirBytes = 1024 * 1024;
// Largest LDS directory image of the flat-LDS form: 160 KiB minus the 16
// waves' candidate scratch (engine.hip FlatScratch<2>, 1536 B each) and 1 KiB.
constexpr size_t kHybLdsDirMaxBytes = 135 * 1024;
// Rounds of candidate loads in flight in the flat-LDS walk: 4 when the
// expected candidates per packet exceed kHybFlat4Candidates (C5: E ≈ 10,
// 0.855 vs 0.895 ms), else 2 (C3: E ≈ 1.3, 0.526 vs 0.541 ms;
// profiles/r1_flat_lds/tune/).  4 rounds need 2560 B of scratch per wave,
// so their directories get kHybFlat4DirBytes.
constexpr double kHybFlat4Candidates = 6.0;
constexpr size_t kHybFlat4DirBytes = 116 * 1024;
// Lane-form directories are two-level: a u32 base per group of 64 buckets +
// a u16 offset per bucket (2.06 B per bucket instead of 4), so the LDS budget
// holds twice the buckets.  A group whose lists exceed 65535 entries keeps
// the whole table on plain u32 directories.
constexpr uint32_t kDir16GroupShift = 6;
// HYBRID LDS directories are two-level with a u32 base per group of 16
// buckets + a u8 offset per bucket (1.25 B per bucket: 1.65x the buckets of
// the u16 form in the same LDS) when every group's lists hold <= 255 entries;
// else the u16 form, else plain u32.  C5: 11.0 -> ~8.5 candidates per packet.
constexpr uint32_t kDir8GroupShift = 4;
// 4-bit form (round 5): one u32 base per group of 16 buckets + a 4-bit count
// per bucket (0.75 B per bucket: 1.67x the buckets of the u8 form in the
// same LDS).  dir[t] = base[t >> 4] + the counts of the group's buckets
// before t, dir[t + 1] = dir[t] + cnt[t]; the counts of group g are the
// dword pair 2g, 2g + 1 of the count array (8-byte aligned), low nibble
// first.  Every bucket list must hold <= 15 entries.
constexpr uint32_t kDir4GroupShift = 4;
// Largest table staged whole in LDS (gfx950: 160 KiB per CU, 1 KiB headroom).
constexpr size_t kLdsTableBytes = 159 * 1024;

enum KeyKind : uint32_t {
    kKeySrc4 = 0,   // IPv4 source address (host-order value of the wire bytes)
    kKeyDst4 = 1,   // IPv4 destination address
    kKeySrc6 = 2,   // IPv6 source address, top 32 bits
    kKeyDst6 = 3,   // IPv6 destination address, top 32 bits
    kKeySport = 4,  // L4 source port
    kKeyDport = 5,  // L4 destination port
    kKeyNone = 6,   // no second key (1-D slot)
};

// Slots per family in the HYBRID global-directory form (nffacl.h NFFACL_MAX_SLOTS).
constexpr uint32_t kMaxSlots = 8;

// Flat-LDS positional forms: the slot parameter block in the LDS image
// (CompiledTable::off_params), kFlatParamDwords per slot s = 0..kMaxSlots-1,
// each word holding the IPv4 value in bits 0..15 and the IPv6 value in 16..31:
//   [0] shift  [1] directory offset  [2] two-level offsets' offset
//   [3] fine 2-D grids: bits2 | shift2 << 8
constexpr uint32_t kFlatParamDwords = 4;
// Packet-side key fields of a slot (kernel key[] order): destination address
// (IPv6: top 32 bits), source address, destination port, source port, zero.
enum SlotField : uint32_t { kFDst = 0, kFSrc = 1, kFDport = 2, kFSport = 3, kFZero = 4 };

}  // namespace nffacl
