// sol.hip — speed-of-light microbenchmarks for the classify access pattern
// (measurement tool, not part of libnffacl).  Every kernel reads n 64-byte
// slots and writes one u32 per slot + one u64 per 64 slots, like
// nffacl_classify_device, but computes only a trivial function of the bytes.
//
//   rows     : lane = packet, 4 x 16 B loads at stride 64 (the classify pattern)
//   rows_pf  : rows + next-batch prefetch (classify's software pipeline)
//   coal     : lane-contiguous 16 B loads (1 KiB per wave instruction), then
//              each packet's dword 3 gathered with ds_bpermute
//   copy     : plain float4 copy n*64 bytes -> n*64 bytes (HBM reference)
//   frames   : packed IMIX frames: per lane its u64 descriptor, then the
//              frame's first 64 bytes (classify_frames' pattern); frames_pf
//              loads the next batch's descriptors + frame lines ahead
//   frames_rs: frames, each wave instruction loading one 16-byte chunk of 64
//              frames' first lines (lane 16r + c: chunk r of frame 16j + c,
//              offsets fetched with ds_bpermute), lanes' frames assembled
//              with permlane row swaps (libnffacl's load_rowswap layout)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../nff-go_amd/csrc/devutil.hpp"

using nffacl::dev::u32x4;
using nffacl::dev::lane_id;

template <bool NT>
__device__ __forceinline__ void ld16(const uint8_t *p, uint32_t (&d)[16]) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u32x4 v = NT ? __builtin_nontemporal_load(q + j) : q[j];
        d[4 * j] = v.x; d[4 * j + 1] = v.y; d[4 * j + 2] = v.z; d[4 * j + 3] = v.w;
    }
}

__device__ __forceinline__ uint32_t fold(const uint32_t (&d)[16]) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) x ^= d[k] * (2 * k + 1);
    return x;
}

template <bool NT>
__global__ void __launch_bounds__(1024) k_rows(const uint8_t *s, uint64_t n, uint32_t *port, uint64_t *bits) {
    const uint32_t lane = lane_id();
    const uint64_t wave0 = uint64_t(blockIdx.x) * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = uint64_t(gridDim.x) * (blockDim.x >> 6) * 64;
    for (uint64_t base = wave0 * 64; base < n; base += step) {
        const uint64_t i = base + lane;
        uint32_t d[16];
        ld16<NT>(s + (i < n ? i : 0) * 64, d);
        const uint32_t r = fold(d);
        if (i < n) port[i] = r;
        const uint64_t b = __builtin_amdgcn_ballot_w64(i < n && (r & 1));
        if (lane == 0) bits[base >> 6] = b;
    }
}

template <bool NT>
__global__ void __launch_bounds__(1024) k_rows_pf(const uint8_t *s, uint64_t n, uint32_t *port, uint64_t *bits) {
    const uint32_t lane = lane_id();
    const uint64_t wave0 = uint64_t(blockIdx.x) * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = uint64_t(gridDim.x) * (blockDim.x >> 6) * 64;
    uint64_t base = wave0 * 64;
    uint32_t d[16];
    if (base < n) ld16<NT>(s + (base + lane < n ? base + lane : 0) * 64, d);
    for (; base < n; base += step) {
        const uint64_t i = base + lane;
        uint32_t cur[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) cur[k] = d[k];
        const uint64_t nb = base + step;
        if (nb < n) ld16<NT>(s + (nb + lane < n ? nb + lane : 0) * 64, d);
        const uint32_t r = fold(cur);
        if (i < n) port[i] = r;
        const uint64_t b = __builtin_amdgcn_ballot_w64(i < n && (r & 1));
        if (lane == 0) bits[base >> 6] = b;
    }
}

__global__ void __launch_bounds__(1024) k_coal(const uint8_t *s, uint64_t n, uint32_t *port, uint64_t *bits) {
    const uint32_t lane = lane_id();
    const uint64_t wave0 = uint64_t(blockIdx.x) * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = uint64_t(gridDim.x) * (blockDim.x >> 6) * 64;
    for (uint64_t base = wave0 * 64; base < n; base += step) {
        // wave's 4 KiB = 4 instructions x 1 KiB contiguous
        const u32x4 *q = reinterpret_cast<const u32x4 *>(s + base * 64);
        uint32_t acc = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const u32x4 v = __builtin_nontemporal_load(q + j * 64 + lane);
            acc ^= v.x * 3 + v.y * 5 + v.z * 7 + v.w * 11;
        }
        // lane l holds chunk (l % 4) of packets (j*16 + l/4): gather one dword per packet
        const uint32_t r = __builtin_amdgcn_ds_bpermute(static_cast<int>((lane & 15) * 4 * 4), static_cast<int>(acc));
        const uint64_t i = base + lane;
        if (i < n) port[i] = r;
        const uint64_t b = __builtin_amdgcn_ballot_w64(i < n && (r & 1));
        if (lane == 0) bits[base >> 6] = b;
    }
}

template <bool PF>
__global__ void __launch_bounds__(1024) k_frames(const uint8_t *fr, const uint64_t *desc, uint64_t n, uint32_t *port,
                                                 uint64_t *bits) {
    const uint32_t lane = lane_id();
    const uint64_t wave0 = uint64_t(blockIdx.x) * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = uint64_t(gridDim.x) * (blockDim.x >> 6) * 64;
    uint32_t nd[16];
    uint64_t nds = 0;
    bool first = true;
    for (uint64_t base = wave0 * 64; base < n; base += step) {
        const uint64_t i = base + lane;
        uint32_t d[16];
        if (!PF || first) {
            const uint64_t ds = i < n ? desc[i] : 0;
            ld16<false>(fr + (ds >> 16), d);
            if (PF) nds = i + step < n ? desc[i + step] : 0;
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) d[k] = nd[k];
        }
        if (PF) {
            if (base + step < n) ld16<false>(fr + (nds >> 16), nd);
            nds = i + 2 * step < n ? desc[i + 2 * step] : 0;
        }
        first = false;
        const uint32_t r = fold(d);
        if (i < n) port[i] = r;
        const uint64_t b = __builtin_amdgcn_ballot_w64(i < n && (r & 1));
        if (lane == 0) bits[base >> 6] = b;
    }
}

__device__ __forceinline__ uint32_t bperm32(uint32_t v, uint32_t src) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(src << 2), static_cast<int>(v)));
}

template <bool NT>
__global__ void __launch_bounds__(1024) k_frames_rs(const uint8_t *fr, const uint64_t *desc, uint64_t n,
                                                    uint32_t *port, uint64_t *bits) {
    const uint32_t lane = lane_id();
    const uint64_t wave0 = uint64_t(blockIdx.x) * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = uint64_t(gridDim.x) * (blockDim.x >> 6) * 64;
    for (uint64_t base = wave0 * 64; base < n; base += step) {
        const uint64_t i = base + lane;
        const uint64_t off = (i < n ? desc[i] : 0) >> 16;
        u32x4 v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t src = 16u * j + (lane & 15u);
            const uint64_t o = uint64_t(bperm32(uint32_t(off), src)) | uint64_t(bperm32(uint32_t(off >> 32), src)) << 32;
            const u32x4 *q = reinterpret_cast<const u32x4 *>(fr + o) + (lane >> 4);
            v[j] = NT ? __builtin_nontemporal_load(q) : *q;
        }
        uint32_t d[16];
        nffacl::dev::rowswap_batch(v, d);
        const uint32_t r = fold(d);
        if (i < n) port[i] = r;
        const uint64_t b = __builtin_amdgcn_ballot_w64(i < n && (r & 1));
        if (lane == 0) bits[base >> 6] = b;
    }
}

__global__ void __launch_bounds__(256) k_copy(const u32x4 *a, u32x4 *b, uint64_t n16) {
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x)
        b[i] = __builtin_nontemporal_load(a + i);
}

extern "C" int sol_run(int which, const void *slots, uint64_t n, void *port, void *bits, void *scratch,
                       int blocks_per_cu, int block, void *stream) {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 g(cus * blocks_per_cu), b(block);
    const uint8_t *s = static_cast<const uint8_t *>(slots);
    uint32_t *p = static_cast<uint32_t *>(port);
    uint64_t *bb = static_cast<uint64_t *>(bits);
    switch (which) {
    case 0: hipLaunchKernelGGL(k_rows<true>, g, b, 0, st, s, n, p, bb); break;
    case 1: hipLaunchKernelGGL(k_rows<false>, g, b, 0, st, s, n, p, bb); break;
    case 2: hipLaunchKernelGGL(k_rows_pf<true>, g, b, 0, st, s, n, p, bb); break;
    case 3: hipLaunchKernelGGL(k_coal, g, b, 0, st, s, n, p, bb); break;
    case 4: hipLaunchKernelGGL(k_copy, g, b, 0, st, reinterpret_cast<const u32x4 *>(slots),
                               static_cast<u32x4 *>(scratch), n * 4); break;
    case 5: hipLaunchKernelGGL(k_frames<false>, g, b, 0, st, s, static_cast<const uint64_t *>(scratch), n, p, bb); break;
    case 6: hipLaunchKernelGGL(k_frames<true>, g, b, 0, st, s, static_cast<const uint64_t *>(scratch), n, p, bb); break;
    case 7: hipLaunchKernelGGL(k_frames_rs<false>, g, b, 0, st, s, static_cast<const uint64_t *>(scratch), n, p, bb); break;
    case 8: hipLaunchKernelGGL(k_frames_rs<true>, g, b, 0, st, s, static_cast<const uint64_t *>(scratch), n, p, bb); break;
    default: return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
