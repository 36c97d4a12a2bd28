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
// The rules of one family are split into "key dimensions".  Each rule is
// assigned to exactly one dimension d and is stored in d's interval index: the
// sorted list of elementary-interval starts of the rules' key ranges on d, and
// per interval the ordered (ascending rule index) candidate list of rules whose
// key range covers that interval.  A packet's first match is the minimum over
// dimensions of the first candidate (in rule order) that passes the full rule
// test, so the index only has to return a superset of the matching rules —
// projections (a non-prefix mask's leading-ones run, the top 32 bits of an
// IPv6 address) keep the result exact.
//
// Dimension header (in the index blob, dwords):
//   [0] key_kind   (kKey*)
//   [1] n_bounds   number of interval starts (>= 1; bounds[0] == 0)
//   [2] radix_bits number of leading key bits used by the radix directory
//   [3] off_radix  dword offset of the radix directory (2^radix_bits + 1 entries)
//   [4] off_bounds dword offset of bounds[n_bounds]   (sorted u32 interval starts)
//   [5] off_lists  dword offset of list_start[n_bounds + 1]
//   [6] off_cands  dword offset of candidates (u32 rule record indices)
//   [7] reserved
constexpr uint32_t kDimHeaderDwords = 8;
enum KeyKind : uint32_t {
    kKeySrc4 = 0,   // IPv4 source address (host-order value of the wire bytes)
    kKeyDst4 = 1,   // IPv4 destination address
    kKeySrc6 = 2,   // IPv6 source address, top 32 bits
    kKeyDst6 = 3,   // IPv6 destination address, top 32 bits
    kKeySport = 4,  // L4 source port
    kKeyDport = 5,  // L4 destination port
};

}  // namespace nffacl
