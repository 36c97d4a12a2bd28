// l2.hpp — L2 ACL engine behind the nffacl_l2engine handle (internal).
//
// The reference's L2 ACL (packet/acl.go:478-491) compares the Ethernet header
// only: destination MAC (wire bytes 0..5), source MAC (6..11) and EtherType
// (12..13), each either exact or ANY (an arbitrary EtherType mask through
// nffacl_l2rules_from_array).  A packet is the four little-endian dwords
// p0..p3 of wire bytes 0..15; a rule is a value v and a mask m over them
// (m3 = EtherType mask in its low 16 bits), matching iff ((p ^ v) & m) == 0.
//
// Two compiled forms, both first-match exact:
//  LINEAR  8-dword records in file order, scanned wave-uniformly:
//            [0..2] v0..v2, [3] v3 | m3 << 16, [4..6] m0..m2, [7] OutputNumber
//  HASH    rules grouped by *shape* (their mask m0..m3); per shape a
//          two-choice cuckoo table keyed by the masked header, holding the
//          first (lowest-index) rule with that key.  A slot is one 16-byte
//          record {k0, k1, k2, k3 | rule index << 16} (k3 = the masked
//          EtherType, 16 bits); an empty slot has rule index 0xFFFF, which
//          never beats a match.  A packet reads both candidate slots of every
//          shape (no probe loop: a key is in one of its two slots or absent)
//          and takes the lowest matching rule index over all shapes — the
//          reference's first match; the OutputNumber comes from a per-rule
//          array after the last shape.  Tables are sized to load <= 1/4; a
//          key set the insertion cannot place (or 0xFFFF+ rules, or more
//          than kL2MaxShapes shapes) compiles LINEAR.
// Rules after the first unconstrained rule (matches everything) are dropped.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <mutex>
#include <vector>

#include "nffacl.h"
#include "rules.hpp"
#include "tables.hpp"

namespace nffacl {

constexpr uint32_t kL2RecDwords = 8;
constexpr uint32_t kL2MaxShapes = 8;
constexpr uint32_t kL2NoRule = 0xFFFFu;  // empty cuckoo slot / no match

struct L2Shape {
    uint32_t m[4];     // header masks of this shape
    uint32_t off;      // dword offset of its cuckoo slots (4 dwords each)
    uint32_t cap_mask; // slots - 1 (power of two)
};

struct L2Compiled {
    int algo = NFFACL_ALGO_LINEAR;
    std::vector<uint32_t> blob;  // LINEAR records, or HASH tables + OutputNumber per rule
    uint32_t n_rules = 0;        // live rules (LINEAR records / output array length)
    uint32_t n_shapes = 0;
    uint32_t off_out = 0;        // HASH: dword offset of the OutputNumber array
    L2Shape shapes[kL2MaxShapes] = {};
};

// Host compilation (AUTO -> HASH when the rules have <= kL2MaxShapes shapes).
L2Compiled compile_l2(const std::vector<nffacl_l2_rule> &eth, int algo);

// Header hashes shared by the host compiler and the kernel: the two cuckoo
// slots of a key are l2_hash & cap_mask and l2_hash_alt(l2_hash) & cap_mask.
// (one multiply each: rotations fold the four header dwords, multiplies and
// shifts mix)
__host__ __device__ inline uint32_t l2_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__host__ __device__ inline uint32_t l2_hash(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    uint32_t h = k0 ^ l2_rotl(k1, 11) ^ l2_rotl(k2, 19) ^ l2_rotl(k3, 27);
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    return h;
}
__host__ __device__ inline uint32_t l2_hash_alt(uint32_t h) {
    h = (h ^ (h >> 16)) * 0x45D9F3Bu;
    return h ^ (h >> 13);
}

// One compiled L2 table resident in HBM (lifetime: tables.hpp).
struct L2Table : DeviceBlob {
    L2Compiled meta;
};
using L2TablePtr = std::shared_ptr<L2Table>;

}  // namespace nffacl

struct nffacl_l2engine {
    int device = 0;
    int num_cus = 256;
    int algo_req = NFFACL_ALGO_AUTO;
    bool coal = true;  // NFFACL_TUNE_L2_COAL (read once at creation): lane-contiguous 64-byte slot loads
    nffacl::TableHome home;  // before `active`: destroyed after it
    std::mutex table_mu;
    nffacl::L2TablePtr active;
    // host path staging (nffacl_l2_classify_host), grown on demand
    std::mutex host_mu;
    hipStream_t stream = nullptr;
    uint8_t *d_slots = nullptr;
    uint32_t *d_port = nullptr;
    size_t cap_bytes = 0, cap_n = 0;
};

namespace nffacl {
int upload_l2(nffacl_l2engine *eng, const nffacl_l2rules &rules, L2TablePtr &out);
int l2_prepare_kernels();
// Both record the launch on `t` (DeviceBlob::note_use).
int l2_launch_slots(nffacl_l2engine *eng, L2Table *t, const uint8_t *d_slots, uint32_t stride,
                    uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream);
int l2_launch_frames(nffacl_l2engine *eng, L2Table *t, const uint8_t *d_frames,
                     const uint64_t *d_desc, uint64_t n, uint32_t *d_port, uint64_t *d_permit,
                     hipStream_t stream);
}  // namespace nffacl
