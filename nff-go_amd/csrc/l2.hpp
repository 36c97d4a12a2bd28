// l2.hpp — L2 ACL engine behind the nffacl_l2engine handle (internal).
//
// The reference's L2 ACL (packet/acl.go:462-491) compares the Ethernet header
// only: destination MAC (wire bytes 0..5), source MAC (6..11) and EtherType
// (12..13).  Compiled form: one 8-dword record per rule in file order,
//   [0..2] value dwords of wire bytes 0..11 (little-endian dwords, pre-masked)
//   [3]    EtherType value (LE 16 of wire bytes 12..13) | its mask << 16
//   [4..6] masks of wire bytes 0..11 (0xff per constrained MAC byte)
//   [7]    OutputNumber
// so a rule matches packet dwords p0..p3 iff
//   ((p0^v0)&m0) | ((p1^v1)&m1) | ((p2^v2)&m2) | ((p3^v3)&(v3>>16)) == 0.
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

// Host compilation of an L2 rule list into device records.
std::vector<uint32_t> compile_l2(const std::vector<nffacl_l2_rule> &eth);

struct L2Table {
    uint32_t *d_rec = nullptr;
    uint32_t n = 0;
    ~L2Table();
};

int upload_l2(int device, const nffacl_l2rules &rules, L2Table *&out);

}  // namespace nffacl

struct nffacl_l2engine {
    int device = 0;
    int num_cus = 256;
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
int l2_launch_slots(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_slots, uint32_t stride,
                    uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream);
int l2_launch_frames(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_frames,
                     const uint64_t *d_desc, uint64_t n, uint32_t *d_port, uint64_t *d_permit,
                     hipStream_t stream);
}  // namespace nffacl
