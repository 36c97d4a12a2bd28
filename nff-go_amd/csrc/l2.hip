// l2.hip — HIP kernels (gfx950) for nff-go's L2 ACL: (*Packet).l2ACL,
// packet/acl.go:478-491, behind L2ACLPort / L2ACLPermit (acl.go:462-476).
//
// One wave64 = 64 consecutive packets, one packet per lane.  Each lane needs
// only the first 16 bytes of its frame (one 16-byte load); the rule records
// are wave-uniform and stream through the scalar data cache, so each rule is
// four masked compares on all 64 packets at once, and a ballot of
// still-undecided lanes ends the scan at the wave's last first-match (the
// reference's `return rule.OutputNumber`).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "devutil.hpp"
#include "l2.hpp"

namespace nffacl {

std::vector<uint32_t> compile_l2(const std::vector<nffacl_l2_rule> &eth) {
    std::vector<uint32_t> rec;
    rec.reserve(eth.size() * kL2RecDwords);
    for (const nffacl_l2_rule &r : eth) {
        uint8_t val[12] = {0}, msk[12] = {0};
        if (r.daddr_not_any) {
            std::memcpy(val, r.daddr, 6);
            std::memset(msk, 0xff, 6);
        }
        if (r.saddr_not_any) {
            std::memcpy(val + 6, r.saddr, 6);
            std::memset(msk + 6, 0xff, 6);
        }
        uint32_t v[3], m[3];
        std::memcpy(v, val, 12);
        std::memcpy(m, msk, 12);
        // (rule.ID ^ SwapBytesUint16(EtherType)) & rule.IDMask  (acl.go:486):
        // the big-endian EtherType compared with ID is, in wire-byte (LE) form,
        // the byte-swapped ID / IDMask.
        const uint32_t em = static_cast<uint32_t>(((r.id_mask & 0xffu) << 8) | (r.id_mask >> 8));
        const uint32_t ev = static_cast<uint32_t>(((r.id & 0xffu) << 8) | (r.id >> 8)) & em;
        const uint32_t w[kL2RecDwords] = {v[0] & m[0], v[1] & m[1], v[2] & m[2], ev | (em << 16),
                                          m[0], m[1], m[2], r.output_number};
        rec.insert(rec.end(), w, w + kL2RecDwords);
        if (!r.daddr_not_any && !r.saddr_not_any && em == 0) break;  // later rules unreachable
    }
    return rec;
}

L2Table::~L2Table() {
    if (d_rec) (void)hipFree(d_rec);
}

int upload_l2(int device, const nffacl_l2rules &rules, L2Table *&out) {
    const std::vector<uint32_t> rec = compile_l2(rules.eth);
    HIP_TRY(hipSetDevice(device));
    L2Table *t = new L2Table();
    t->n = static_cast<uint32_t>(rec.size() / kL2RecDwords);
    // at least one record so the device pointer is always valid
    const size_t bytes = std::max<size_t>(rec.size(), kL2RecDwords) * sizeof(uint32_t);
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&t->d_rec), bytes);
    if (e == hipSuccess) e = hipMemset(t->d_rec, 0, bytes);
    if (e == hipSuccess && !rec.empty())
        e = hipMemcpy(t->d_rec, rec.data(), rec.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_last_error(std::string("L2 table upload: ") + hipGetErrorString(e));
        delete t;
        return NFFACL_ERR_HIP;
    }
    out = t;
    return NFFACL_OK;
}

namespace dev {

__device__ __forceinline__ uint32_t classify_l2(const uint32_t (&p)[4], bool live,
                                                const uint32_t *__restrict__ rec, uint32_t n) {
    uint32_t res = 0;
    bool pend = live;
    for (uint32_t r = 0; r < n; ++r) {
        const uint32_t *R = rec + r * kL2RecDwords;
        const uint32_t m = ((p[0] ^ R[0]) & R[4]) | ((p[1] ^ R[1]) & R[5]) | ((p[2] ^ R[2]) & R[6]) |
                           ((p[3] ^ R[3]) & (R[3] >> 16));
        const bool take = pend && m == 0u;
        if (ballot(take)) {
            if (take) { res = R[7]; pend = false; }
            if (!ballot(pend)) break;
        }
    }
    return res;
}

__global__ void __launch_bounds__(256)
k_l2_slots(const uint8_t *__restrict__ slots, uint32_t stride, uint64_t n, const uint32_t *__restrict__ rec,
           uint32_t nrec, uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    NFFACL_WAVE_LOOP(n) {
        const uint64_t idx = base + lane;
        const bool live = idx < n;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(slots + (live ? idx : 0) * stride);
        const uint32_t p[4] = {v.x, v.y, v.z, v.w};
        store_verdicts(base, lane, live, classify_l2(p, live, rec, nrec), port_out, permit_out);
    }
}

// Packed frames: desc = offset << 16 | length; bytes >= length read as 0.
__global__ void __launch_bounds__(256)
k_l2_frames(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint64_t n,
            const uint32_t *__restrict__ rec, uint32_t nrec, uint32_t *__restrict__ port_out,
            uint64_t *__restrict__ permit_out) {
    NFFACL_WAVE_LOOP(n) {
        const uint64_t idx = base + lane;
        const bool live = idx < n;
        const uint64_t ds = live ? desc[idx] : 0;
        const u32x4 v = *reinterpret_cast<const u32x4 *>(frames + (ds >> 16));
        uint32_t p[4] = {v.x, v.y, v.z, v.w};
        clip_dwords<4>(p, static_cast<uint32_t>(ds & 0xFFFFu));
        store_verdicts(base, lane, live, classify_l2(p, live, rec, nrec), port_out, permit_out);
    }
}

}  // namespace dev

static uint32_t l2_grid(const nffacl_l2engine *eng, uint64_t n, uint32_t block) {
    const uint64_t blocks_needed = ((n + 63) / 64 * 64 + block - 1) / block;
    const uint64_t cap = uint64_t(eng->num_cus) * 8;
    return static_cast<uint32_t>(std::max<uint64_t>(1, std::min(blocks_needed, cap)));
}

int l2_launch_slots(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_slots, uint32_t stride,
                    uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream) {
    if (n == 0) return NFFACL_OK;
    constexpr uint32_t block = 256;
    hipLaunchKernelGGL(dev::k_l2_slots, dim3(l2_grid(eng, n, block)), dim3(block), 0, stream, d_slots, stride, n,
                       t->d_rec, t->n, d_port, d_permit);
    HIP_TRY(hipGetLastError());
    return NFFACL_OK;
}

int l2_launch_frames(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_frames, const uint64_t *d_desc,
                     uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream) {
    if (n == 0) return NFFACL_OK;
    constexpr uint32_t block = 256;
    hipLaunchKernelGGL(dev::k_l2_frames, dim3(l2_grid(eng, n, block)), dim3(block), 0, stream, d_frames, d_desc,
                       n, t->d_rec, t->n, d_port, d_permit);
    HIP_TRY(hipGetLastError());
    return NFFACL_OK;
}

}  // namespace nffacl
