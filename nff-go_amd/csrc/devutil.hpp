// devutil.hpp — device helpers shared by the L3 (engine.hip) and L2 (l2.hip)
// kernels of libnffacl (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace nffacl {

void set_last_error(const std::string &s);

namespace dev {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Zero the bytes of d[] at or past `len`.
template <int N>
__device__ __forceinline__ void clip_dwords(uint32_t (&d)[N], uint32_t len) {
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int rem = static_cast<int>(len) - 4 * k;  // valid bytes in dword k
        const uint32_t keep = rem >= 4 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << (8 * rem)) - 1u));
        d[k] &= keep;
    }
}
__device__ __forceinline__ void clip16(uint32_t (&d)[16], uint32_t len) { clip_dwords<16>(d, len); }

// Port vector (u32 per packet) + permit bitmap (one 64-bit ballot per wave).
__device__ __forceinline__ void store_verdicts(uint64_t base, uint32_t lane, bool live, uint32_t res,
                                               uint32_t *__restrict__ port_out,
                                               uint64_t *__restrict__ permit_out) {
    if (live && port_out) port_out[base + lane] = res;
    const uint64_t permit = ballot(live && res != 0u);
    if (permit_out && lane == 0) permit_out[base >> 6] = permit;
}

}  // namespace dev
}  // namespace nffacl

// One wave = 64 consecutive packets per grid-stride step.
#define NFFACL_WAVE_LOOP(n)                                                                   \
    const uint32_t lane = ::nffacl::dev::lane_id();                                           \
    const uint32_t wpb = blockDim.x >> 6;                                                     \
    const uint64_t wave0 = uint64_t(blockIdx.x) * wpb +                                       \
                           __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);                  \
    const uint64_t nwaves = uint64_t(gridDim.x) * wpb;                                        \
    for (uint64_t base = wave0 * 64; base < (n); base += nwaves * 64)

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) {                                                          \
            ::nffacl::set_last_error(std::string(#expr) + ": " + hipGetErrorString(e_));  \
            return NFFACL_ERR_HIP;                                                       \
        }                                                                                \
    } while (0)
