// v127_probe — is a VALU result in v127 (the last register of a 128-VGPR
// allocation, 4 waves per SIMD filling the 512-entry file) read back intact?
// DESIGN.md §4.3 (round 6): the NS = 7 pipelined walk lost IPv6 matches
// only where the compiler kept the destination prefix length in v127
// (v_min_u32_sdwa v127 ... BYTE_1, read 10 instructions later by
// v_lshrrev_b64 v[..], v127, s[..]), more often the more waves per SIMD.
// Each variant repeats one fixed inline-asm sequence (no compiler
// scheduling inside it) on every thread of 1024-thread workgroups and counts
// results that differ from the same arithmetic done in C:
//   0  SDWA v_min_u32 -> v127, ds_bpermute + lgkmcnt wait, v_lshrrev_b64 reads v127
//   1  the same with v125 (register control)
//   2  v_bfe_u32 + v_min_u32 (no SDWA) -> v127, same read (SDWA control)
//   3  SDWA -> v127, read by v_mov_b32 (32-bit read control)
// usage: v127_probe [iters]  -> one JSON line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));      \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

template <int VAR>
__global__ void __launch_bounds__(1024) k_probe(uint32_t seed, uint32_t iters, unsigned long long *bad) {
    uint32_t x = seed ^ (blockIdx.x * 1024u + threadIdx.x) * 2654435761u;
    const uint32_t c = 32u;
    const uint64_t m = 0xFFFFFFFF00000000ull;
    const uint32_t addr = ((threadIdx.x + 1u) & 63u) << 2;
    uint32_t errs = 0;
    for (uint32_t it = 0; it < iters; ++it) {
        x = x * 1664525u + 1013904223u;
        uint64_t o = 0;
        uint32_t t = 0;
        if constexpr (VAR == 0) {
            asm volatile(
                "v_min_u32_sdwa v127, %[x], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n\t"
                "ds_bpermute_b32 %[t], %[a], %[x]\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "v_lshrrev_b64 %[o], v127, %[m]"
                : [o] "=&v"(o), [t] "=&v"(t)
                : [x] "v"(x), [c] "v"(c), [a] "v"(addr), [m] "s"(m)
                : "v127", "memory");
        } else if constexpr (VAR == 1) {
            asm volatile(
                "v_min_u32_sdwa v125, %[x], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n\t"
                "ds_bpermute_b32 %[t], %[a], %[x]\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "v_lshrrev_b64 %[o], v125, %[m]"
                : [o] "=&v"(o), [t] "=&v"(t)
                : [x] "v"(x), [c] "v"(c), [a] "v"(addr), [m] "s"(m)
                : "v125", "v127", "memory");
        } else if constexpr (VAR == 2) {
            asm volatile(
                "v_bfe_u32 v127, %[x], 8, 8\n\t"
                "v_min_u32_e32 v127, v127, %[c]\n\t"
                "ds_bpermute_b32 %[t], %[a], %[x]\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "v_lshrrev_b64 %[o], v127, %[m]"
                : [o] "=&v"(o), [t] "=&v"(t)
                : [x] "v"(x), [c] "v"(c), [a] "v"(addr), [m] "s"(m)
                : "v127", "memory");
        } else {
            uint32_t r = 0;
            asm volatile(
                "v_min_u32_sdwa v127, %[x], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n\t"
                "ds_bpermute_b32 %[t], %[a], %[x]\n\t"
                "s_waitcnt lgkmcnt(0)\n\t"
                "v_mov_b32 %[r], v127"
                : [r] "=&v"(r), [t] "=&v"(t)
                : [x] "v"(x), [c] "v"(c), [a] "v"(addr)
                : "v127", "memory");
            o = m >> r;
        }
        const uint32_t len = min((x >> 8) & 0xFFu, c);
        errs += o != (m >> len) ? 1u : 0u;
        x ^= t;  // keep the bpermute live
    }
    if (errs) atomicAdd(bad, static_cast<unsigned long long>(errs));
}

int main(int argc, char **argv) {
    const uint32_t iters = argc > 1 ? static_cast<uint32_t>(std::atoi(argv[1])) : 4096u;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long *d_bad = nullptr;
    CHECK(hipMalloc(&d_bad, 4 * sizeof(unsigned long long)));
    CHECK(hipMemset(d_bad, 0, 4 * sizeof(unsigned long long)));
    const dim3 grid(cus * 4), block(1024);
    for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(k_probe<0>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 0);
        hipLaunchKernelGGL(k_probe<1>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 1);
        hipLaunchKernelGGL(k_probe<2>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 2);
        hipLaunchKernelGGL(k_probe<3>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 3);
    }
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    unsigned long long bad[4];
    CHECK(hipMemcpy(bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
    const double per = 4.0 * double(grid.x) * block.x * iters;
    std::printf("{\"ops_per_variant\": %.0f, \"bad\": {\"sdwa_v127_b64\": %llu, \"sdwa_v125_b64\": %llu, "
                "\"bfe_v127_b64\": %llu, \"sdwa_v127_mov\": %llu}}\n",
                per, bad[0], bad[1], bad[2], bad[3]);
    return 0;
}
