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

// ---- lane-contiguous batch load for 64-byte slots (a wave's 64 packets =
// 4 KiB contiguous) ---------------------------------------------------------
// Row-swap variant (MODE 4): lane l = 16r + c loads, for instruction j, the
// 16 bytes at 1024j + 64c + 16r — chunk r of packet 16j + c; every
// instruction still covers one contiguous KiB.  Register j of row r then holds
// M[r][j] = chunk r of packet 16j + c, and a 4x4 transpose across the four
// 16-lane rows (v_permlane16_swap on register pairs (0,1), (2,3), then
// v_permlane32_swap on (0,2), (1,3): 4 instructions per dword plane) leaves
// register m of row r = chunk m of packet 16r + c = packet `lane` — no
// per-lane packet remap, no permit re-order.
template <bool NT>
__device__ __forceinline__ void load_rowswap(const uint8_t *__restrict__ wave_base, uint32_t lane, u32x4 (&v)[4]) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(wave_base) + 4u * (lane & 15u) + (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = NT ? __builtin_nontemporal_load(q + 64 * j) : q[64 * j];
}

__device__ __forceinline__ void rowswap_batch(const u32x4 (&v)[4], uint32_t (&d)[16]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // dword plane k of every chunk
        uint32_t a0 = v[0][k], a1 = v[1][k], a2 = v[2][k], a3 = v[3][k];
        const auto p01 = __builtin_amdgcn_permlane16_swap(a0, a1, false, false);
        const auto p23 = __builtin_amdgcn_permlane16_swap(a2, a3, false, false);
        const auto q02 = __builtin_amdgcn_permlane32_swap(p01[0], p23[0], false, false);
        const auto q13 = __builtin_amdgcn_permlane32_swap(p01[1], p23[1], false, false);
        d[0 + k] = q02[0];
        d[4 + k] = q13[0];
        d[8 + k] = q02[1];
        d[12 + k] = q13[1];
    }
}

// Chunk 0 (bytes 0..15) of packet `lane` only: 3 of rowswap_batch's 4 swaps
// per dword plane (the L2 kernel's Ethernet header).
__device__ __forceinline__ void rowswap_chunk0(const u32x4 (&v)[4], uint32_t (&d)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const auto p01 = __builtin_amdgcn_permlane16_swap(v[0][k], v[1][k], false, false);
        const auto p23 = __builtin_amdgcn_permlane16_swap(v[2][k], v[3][k], false, false);
        d[k] = __builtin_amdgcn_permlane32_swap(p01[0], p23[0], false, false)[0];
    }
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

// A verdict store, nontemporal where the kernel gathers an L2-sized table
// (NT): a C5 launch writes 64 MiB of ports through L2, where the ~4 MB of
// rule entries want to stay — 0.5046 / 0.4958 vs 0.5103 / 0.5116 ms; the
// streaming kernels (C2 0.2090 vs 0.2047, C3 0.4084 vs 0.4048 ms) keep plain
// stores (profiles/r6_ab/nt/).
template <bool NT>
__device__ __forceinline__ void store_port(uint32_t *p, uint32_t v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

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
