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
//  HASH    rules grouped by *shape* (their mask m0..m3); per shape an
//          open-addressing table keyed by the masked header, holding the
//          first (lowest-index) rule with that key.  A packet probes every
//          shape whose first rule precedes its best match so far; the answer
//          is the lowest rule index found — the reference's first match.
//          Buckets of four slots (load <= 1/2): a bucket is four 32-bit
//          fingerprints (key hash | 1; 0 = empty) read with one 16-byte load,
//          and in a parallel array one 8-dword key record per slot
//          {k0..k3, rule index, OutputNumber, 0, 0} read only on a
//          fingerprint match.  A lookup almost always ends in its first
//          bucket (a match, or a free slot proving absence).
// Rules after the first unconstrained rule (matches everything) are dropped.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <vector>

#include "nffacl.h"
#include "rules.hpp"

namespace nffacl {

constexpr uint32_t kL2RecDwords = 8;
constexpr uint32_t kL2BucketSlots = 4;
constexpr uint32_t kL2KeyDwords = 8;
constexpr uint32_t kL2MaxShapes = 8;

struct L2Shape {
    uint32_t m[4];     // header masks of this shape
    uint32_t off;      // dword offset of its fingerprint buckets (4 dwords each)
    uint32_t cap_mask; // buckets - 1 (power of two)
    uint32_t first;    // lowest rule index of the shape
    uint32_t off_key;  // dword offset of its key records (8 dwords per slot)
};

struct L2Compiled {
    int algo = NFFACL_ALGO_LINEAR;
    std::vector<uint32_t> blob;  // LINEAR records or HASH tables
    uint32_t n_rules = 0;        // live rules (LINEAR records)
    uint32_t n_shapes = 0;
    L2Shape shapes[kL2MaxShapes] = {};
};

// Host compilation (AUTO -> HASH when the rules have <= kL2MaxShapes shapes).
L2Compiled compile_l2(const std::vector<nffacl_l2_rule> &eth, int algo);

// Header hash shared by the host compiler and the kernel.
// (one multiply: rotations fold the four header dwords, the multiply and
// shifts mix; collisions cost probes, never correctness)
__host__ __device__ inline uint32_t l2_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__host__ __device__ inline uint32_t l2_hash(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    uint32_t h = k0 ^ l2_rotl(k1, 11) ^ l2_rotl(k2, 19) ^ l2_rotl(k3, 27);
    h ^= h >> 16;
    h *= 0x7FEB352Du;
    h ^= h >> 15;
    return h;
}

struct L2Table {
    uint32_t *d_blob = nullptr;
    L2Compiled meta;
    ~L2Table();
};

int upload_l2(int device, const nffacl_l2rules &rules, int algo, L2Table *&out);

}  // namespace nffacl

struct nffacl_l2engine {
    int device = 0;
    int num_cus = 256;
    int algo_req = NFFACL_ALGO_AUTO;
    std::mutex table_mu;
    nffacl::L2Table *active = nullptr;
    nffacl::L2Table *retired = nullptr;
    // host path staging (nffacl_l2_classify_host), grown on demand
    std::mutex host_mu;
    hipStream_t stream = nullptr;
    uint8_t *d_slots = nullptr;
    uint32_t *d_port = nullptr;
    size_t cap_bytes = 0, cap_n = 0;
};

namespace nffacl {
int l2_prepare_kernels();
int l2_launch_slots(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_slots, uint32_t stride,
                    uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream);
int l2_launch_frames(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_frames,
                     const uint64_t *d_desc, uint64_t n, uint32_t *d_port, uint64_t *d_permit,
                     hipStream_t stream);
}  // namespace nffacl
