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
//   4  the failing kernel's IPv6-test block verbatim (v115..v127)
//   5  the same block two registers lower (v113..v125)
//   6  block 4 with no ds_bpermute returning into v126 (that one into v114)
//   7  block 4 with v127 written by v_bfe_u32 + v_min_u32 (no SDWA)
//   8  block 4 with every ds_bpermute returned (lgkmcnt(0)) before the v127 write
//   9  v0 = -1 in every wave, v_lshrrev_b64 with its 32-bit shift amount in v127
//  10  the same with the shift amount in v125
//  11  the same as 9 with a 32-bit shift (v_lshrrev_b32) reading v127
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


// Variants 4 / 5: the failing kernel's IPv6-test block instruction for
// instruction (k_indexed_slots<7,11,4>, registers v115..v127 as compiled),
// and the same block two registers lower (v113..v125, as the exact NS = 6
// kernel allocates it).  Checks the destination prefix length (v127 / v125)
// and the mask shifted by it.
#define BLOCK(R115, R116, R117, R118, R119, R120, R121, R122, R123, R124, R125, R126, R127, P116_117)         \
    "v_lshlrev_b32 " R116 ", 2, %[own]\n\t"                                                                      \
    "ds_bpermute_b32 " R126 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R120 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R122 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R124 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R125 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R118 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R119 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R121 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R123 ", " R116 ", %[x]\n\t"                                                              \
    "v_add_u32_e32 " R116 ", %[sa], %[own]\n\t"                                                                 \
    "v_cmp_gt_u32_e32 vcc, %[sa], " R116 "\n\t"                                                                 \
    "v_min_u32_sdwa " R116 ", %[lens], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD\n\t" \
    "v_xor_b32_e32 " R115 ", %[own], %[x]\n\t"                                                                  \
    "v_bfe_i32 " R117 ", %[x], 8, 1\n\t"                                                                        \
    "s_waitcnt lgkmcnt(8)\n\t"                                                                                  \
    "v_pk_max_u16 %[t0], " R126 ", %[t0]\n\t"                                                                   \
    "v_min_u32_sdwa " R127 ", %[lens], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n\t" \
    "v_bitop3_b32 " R115 ", " R115 ", %[sa], " R117 " bitop3:0x80\n\t"                                         \
    "v_lshrrev_b64 " P116_117 ", " R116 ", %[m]\n\t"                                                            \
    "v_pk_min_u16 %[t0], %[t0], %[x]\n\t"                                                                       \
    "s_waitcnt lgkmcnt(7)\n\t"                                                                                  \
    "v_xor_b32_e32 %[t1], " R120 ", %[x]\n\t"                                                                   \
    "s_waitcnt lgkmcnt(6)\n\t"                                                                                  \
    "v_xor_b32_e32 %[t1], " R122 ", %[t1]\n\t"                                                                  \
    "s_waitcnt lgkmcnt(5)\n\t"                                                                                  \
    "v_bitop3_b32 %[t2], " R124 ", " R116 ", %[x] bitop3:0x48\n\t"                                             \
    "v_lshrrev_b64 " P116_117 ", " R127 ", %[m]\n\t"                                                            \
    "v_ffbh_u32_e32 %[t1], %[t1]\n\t"                                                                           \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                                  \
    "v_mov_b32 %[r0], " R127 "\n\t"                                                                             \
    "v_mov_b32 %[r1], " R116 "\n\t"

#define BLOCK_E(R115, R116, R117, R118, R119, R120, R121, R122, R123, R124, R125, R126, R127, P116_117)         \
    "v_lshlrev_b32 " R116 ", 2, %[own]\n\t"                                                                      \
    "ds_bpermute_b32 " R126 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R120 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R122 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R124 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R125 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R118 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R119 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R121 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R123 ", " R116 ", %[x]\n\t"                                                              \
    "v_add_u32_e32 " R116 ", %[sa], %[own]\n\t"                                                                 \
    "v_cmp_gt_u32_e32 vcc, %[sa], " R116 "\n\t"                                                                 \
    "v_min_u32_sdwa " R116 ", %[lens], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD\n\t" \
    "v_xor_b32_e32 " R115 ", %[own], %[x]\n\t"                                                                  \
    "v_bfe_i32 " R117 ", %[x], 8, 1\n\t"                                                                        \
    "s_waitcnt lgkmcnt(8)\n\t"                                                                                  \
    "v_pk_max_u16 %[t0], " R126 ", %[t0]\n\t"                                                                   \
    "v_bfe_u32 " R127 ", %[lens], 8, 8\n\t"                                                                  \
    "v_min_u32_e32 " R127 ", " R127 ", %[c]\n\t"                                                               \
    "v_bitop3_b32 " R115 ", " R115 ", %[sa], " R117 " bitop3:0x80\n\t"                                         \
    "v_lshrrev_b64 " P116_117 ", " R116 ", %[m]\n\t"                                                            \
    "v_pk_min_u16 %[t0], %[t0], %[x]\n\t"                                                                       \
    "s_waitcnt lgkmcnt(7)\n\t"                                                                                  \
    "v_xor_b32_e32 %[t1], " R120 ", %[x]\n\t"                                                                   \
    "s_waitcnt lgkmcnt(6)\n\t"                                                                                  \
    "v_xor_b32_e32 %[t1], " R122 ", %[t1]\n\t"                                                                  \
    "s_waitcnt lgkmcnt(5)\n\t"                                                                                  \
    "v_bitop3_b32 %[t2], " R124 ", " R116 ", %[x] bitop3:0x48\n\t"                                             \
    "v_lshrrev_b64 " P116_117 ", " R127 ", %[m]\n\t"                                                            \
    "v_ffbh_u32_e32 %[t1], %[t1]\n\t"                                                                           \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                                  \
    "v_mov_b32 %[r0], " R127 "\n\t"                                                                             \
    "v_mov_b32 %[r1], " R116 "\n\t"

#define BLOCK_F(R115, R116, R117, R118, R119, R120, R121, R122, R123, R124, R125, R126, R127, P116_117)         \
    "v_lshlrev_b32 " R116 ", 2, %[own]\n\t"                                                                      \
    "ds_bpermute_b32 " R126 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R120 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R122 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R124 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R125 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R118 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R119 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R121 ", " R116 ", %[x]\n\t"                                                              \
    "ds_bpermute_b32 " R123 ", " R116 ", %[x]\n\t"                                                              \
    "v_add_u32_e32 " R116 ", %[sa], %[own]\n\t"                                                                 \
    "v_cmp_gt_u32_e32 vcc, %[sa], " R116 "\n\t"                                                                 \
    "v_min_u32_sdwa " R116 ", %[lens], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD\n\t" \
    "v_xor_b32_e32 " R115 ", %[own], %[x]\n\t"                                                                  \
    "v_bfe_i32 " R117 ", %[x], 8, 1\n\t"                                                                        \
    "s_waitcnt lgkmcnt(8)\n\t"                                                                                  \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                                  \
    "v_pk_max_u16 %[t0], " R126 ", %[t0]\n\t"                                                                   \
    "v_min_u32_sdwa " R127 ", %[lens], %[c] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n\t" \
    "v_bitop3_b32 " R115 ", " R115 ", %[sa], " R117 " bitop3:0x80\n\t"                                         \
    "v_lshrrev_b64 " P116_117 ", " R116 ", %[m]\n\t"                                                            \
    "v_pk_min_u16 %[t0], %[t0], %[x]\n\t"                                                                       \
    "s_waitcnt lgkmcnt(7)\n\t"                                                                                  \
    "v_xor_b32_e32 %[t1], " R120 ", %[x]\n\t"                                                                   \
    "s_waitcnt lgkmcnt(6)\n\t"                                                                                  \
    "v_xor_b32_e32 %[t1], " R122 ", %[t1]\n\t"                                                                  \
    "s_waitcnt lgkmcnt(5)\n\t"                                                                                  \
    "v_bitop3_b32 %[t2], " R124 ", " R116 ", %[x] bitop3:0x48\n\t"                                             \
    "v_lshrrev_b64 " P116_117 ", " R127 ", %[m]\n\t"                                                            \
    "v_ffbh_u32_e32 %[t1], %[t1]\n\t"                                                                           \
    "s_waitcnt lgkmcnt(0)\n\t"                                                                                  \
    "v_mov_b32 %[r0], " R127 "\n\t"                                                                             \
    "v_mov_b32 %[r1], " R116 "\n\t"

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
        } else if constexpr (VAR >= 9) {
            // v0 = -1 in every wave, then a 64-bit shift whose 32-bit shift
            // amount sits in v127 (9), v125 (10), or a 32-bit shift reading
            // v127 (11): does the read of the top register see past it?
            const uint32_t sh = (x >> 8) & 31u;
            uint32_t o32 = 0;
            if constexpr (VAR == 9)
                asm volatile("v_mov_b32 v0, -1\n\tv_mov_b32 v127, %[sh]\n\ts_nop 4\n\tv_lshrrev_b64 %[o], v127, %[m]"
                             : [o] "=&v"(o) : [sh] "v"(sh), [m] "s"(m) : "v0", "v127");
            else if constexpr (VAR == 10)
                asm volatile("v_mov_b32 v0, -1\n\tv_mov_b32 v125, %[sh]\n\ts_nop 4\n\tv_lshrrev_b64 %[o], v125, %[m]"
                             : [o] "=&v"(o) : [sh] "v"(sh), [m] "s"(m) : "v0", "v125", "v127");
            else
                asm volatile("v_mov_b32 v0, -1\n\tv_mov_b32 v127, %[sh]\n\ts_nop 4\n\tv_lshrrev_b32 %[o], v127, %[x]"
                             : [o] "=&v"(o32) : [sh] "v"(sh), [x] "v"(0xFFFFFFFFu) : "v0", "v127");
            if constexpr (VAR == 11) errs += o32 != (0xFFFFFFFFu >> sh) ? 1u : 0u;
            else errs += o != (m >> sh) ? 1u : 0u;
            continue;
        } else if constexpr (VAR >= 4) {
            uint32_t r0 = 0, r1 = 0, t0 = x, t1 = 0, t2 = 0;
            const uint32_t own = (threadIdx.x + 7u) & 63u, lens = x;
            if constexpr (VAR == 4) {
                asm volatile(BLOCK("v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124",
                                   "v125", "v126", "v127", "v[116:117]")
                             : [r0] "=&v"(r0), [r1] "=&v"(r1), [t0] "+&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
                             : [x] "v"(x), [own] "v"(own), [lens] "v"(lens), [c] "v"(c), [sa] "s"(seed), [m] "s"(m)
                             : "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125",
                               "v126", "v127", "vcc", "memory");
            } else if constexpr (VAR == 6) {  // no DS return into v126
                asm volatile(BLOCK("v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124",
                                   "v125", "v114", "v127", "v[116:117]")
                             : [r0] "=&v"(r0), [r1] "=&v"(r1), [t0] "+&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
                             : [x] "v"(x), [own] "v"(own), [lens] "v"(lens), [c] "v"(c), [sa] "s"(seed), [m] "s"(m)
                             : "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124",
                               "v125", "v126", "v127", "vcc", "memory");
            } else if constexpr (VAR == 7) {  // v127 by plain VALU (no SDWA)
                asm volatile(BLOCK_E("v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124",
                                     "v125", "v126", "v127", "v[116:117]")
                             : [r0] "=&v"(r0), [r1] "=&v"(r1), [t0] "+&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
                             : [x] "v"(x), [own] "v"(own), [lens] "v"(lens), [c] "v"(c), [sa] "s"(seed), [m] "s"(m)
                             : "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125",
                               "v126", "v127", "vcc", "memory");
            } else if constexpr (VAR == 8) {  // every bpermute returned before the v127 write
                asm volatile(BLOCK_F("v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124",
                                     "v125", "v126", "v127", "v[116:117]")
                             : [r0] "=&v"(r0), [r1] "=&v"(r1), [t0] "+&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
                             : [x] "v"(x), [own] "v"(own), [lens] "v"(lens), [c] "v"(c), [sa] "s"(seed), [m] "s"(m)
                             : "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123", "v124", "v125",
                               "v126", "v127", "vcc", "memory");
            } else {  // VAR == 5
                asm volatile(BLOCK("v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",
                                   "v123", "v124", "v125", "v[114:115]")
                             : [r0] "=&v"(r0), [r1] "=&v"(r1), [t0] "+&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
                             : [x] "v"(x), [own] "v"(own), [lens] "v"(lens), [c] "v"(c), [sa] "s"(seed), [m] "s"(m)
                             : "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122", "v123",
                               "v124", "v125", "v127", "vcc", "memory");
            }
            const uint32_t dl = min((lens >> 8) & 0xFFu, c);
            errs += (r0 != dl) || (r1 != static_cast<uint32_t>(m >> dl)) ? 1u : 0u;
            x ^= t0 ^ t1 ^ t2;
            continue;
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
    CHECK(hipMalloc(&d_bad, 12 * sizeof(unsigned long long)));
    CHECK(hipMemset(d_bad, 0, 12 * sizeof(unsigned long long)));
    const dim3 grid(cus * 4), block(1024);
    for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(k_probe<0>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 0);
        hipLaunchKernelGGL(k_probe<1>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 1);
        hipLaunchKernelGGL(k_probe<2>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 2);
        hipLaunchKernelGGL(k_probe<3>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 3);
        hipLaunchKernelGGL(k_probe<4>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 4);
        hipLaunchKernelGGL(k_probe<5>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 5);
        hipLaunchKernelGGL(k_probe<6>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 6);
        hipLaunchKernelGGL(k_probe<7>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 7);
        hipLaunchKernelGGL(k_probe<8>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 8);
        hipLaunchKernelGGL(k_probe<9>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 9);
        hipLaunchKernelGGL(k_probe<10>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 10);
        hipLaunchKernelGGL(k_probe<11>, grid, block, 0, 0, 1234u + rep, iters, d_bad + 11);
    }
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    unsigned long long bad[12];
    CHECK(hipMemcpy(bad, d_bad, sizeof bad, hipMemcpyDeviceToHost));
    const double per = 4.0 * double(grid.x) * block.x * iters;
    std::printf("{\"ops_per_variant\": %.0f, \"bad\": {\"sdwa_v127_b64\": %llu, \"sdwa_v125_b64\": %llu, "
                "\"bfe_v127_b64\": %llu, \"sdwa_v127_mov\": %llu, \"ns7_block_v127\": %llu, "
                "\"ns7_block_v125\": %llu, \"block_no_ds_into_v126\": %llu, \"block_v127_plain_valu\": %llu, "
                "\"block_ds_drained_first\": %llu, \"v0m1_shift64_v127\": %llu, \"v0m1_shift64_v125\": %llu, "
                "\"v0m1_shift32_v127\": %llu}}\n",
                per, bad[0], bad[1], bad[2], bad[3], bad[4], bad[5], bad[6], bad[7], bad[8], bad[9], bad[10], bad[11]);
    return 0;
}
