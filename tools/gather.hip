// gather.hip — microbenchmark (measurement tool, not part of libnffacl): the
// cost of per-lane random table reads by the number of distinct cache lines
// one wave instruction touches, from an L2-resident table, against LDS.
//
//   hipcc --offload-arch=gfx950 -O3 -o gather tools/gather.hip && ./gather
//
// Each wave issues ITERS independent-address load instructions (4 in flight
// per dependency step); lanes are grouped so that one instruction touches K
// distinct 128-byte lines (64/K lanes share a line).  Prints ns per wave
// instruction per CU = kernel time * CUs / (waves * ITERS).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
            return 1;                                                                \
        }                                                                            \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 256;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    return x;
}

// W = 1: 4-byte loads, W = 4: 16-byte loads.  lines: table size in 128-B lines (power of 2).
template <int W>
__global__ void __launch_bounds__(1024) k_gather(const uint32_t *__restrict__ tab, uint32_t lines, uint32_t k,
                                                 uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t grp = lane / (64u / k);  // lanes of a group share a line
    const uint32_t sub = lane % (64u / k);  // position inside the line
    uint32_t acc = 0, seed = wave * 7919u;
    for (int i = 0; i < ITERS; i += 4) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t line = mix(seed + (i + j) * 131u + grp * 977u + acc * 0u) & (lines - 1u);
            const uint32_t dw = line * 32u + (sub * W) % 32u;
            if (W == 4) {
                const u32x4 q = *reinterpret_cast<const u32x4 *>(tab + dw);
                v[j] = q.x ^ q.y ^ q.z ^ q.w;
            } else {
                v[j] = tab[dw];
            }
        }
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        seed ^= acc & 1u;  // a dependency per 4 loads
    }
    if (acc == 0x12345678u) out[wave] = acc;
}

// 24-byte entries at random entry numbers (the flat walk's candidate loads):
// PAIR = 0: each lane one entry, words 0..2 and 3..5 (dwordx4 + dwordx2);
// PAIR = 1: two lanes per entry, each one 12-byte half (one dwordx3), so one
// instruction covers 32 entries.  Timed per 64 entries.
typedef uint32_t u32x3 __attribute__((ext_vector_type(3), aligned(4)));
template <int PAIR>
__global__ void __launch_bounds__(1024) k_ent24(const uint32_t *__restrict__ tab, uint32_t ents, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    uint32_t acc = 0, seed = wave * 7919u;
    for (int i = 0; i < ITERS; i += 4) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (PAIR) {
                // instruction j covers entries of 32 lane pairs
                const uint32_t e = mix(seed + (i + j) * 131u + (lane >> 1) * 977u) % ents;
                const u32x3 q = *reinterpret_cast<const u32x3 *>(tab + e * 6u + 3u * (lane & 1u));
                v[j] = q.x ^ q.y ^ q.z;
            } else {
                const uint32_t e = mix(seed + (i + j) * 131u + lane * 977u) % ents;
                const u32x3 a = *reinterpret_cast<const u32x3 *>(tab + e * 6u);
                const u32x3 b = *reinterpret_cast<const u32x3 *>(tab + e * 6u + 3u);
                v[j] = a.x ^ a.y ^ a.z ^ b.x ^ b.y ^ b.z;
            }
        }
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        seed ^= acc & 1u;
    }
    if (acc == 0x12345678u) out[wave] = acc;
}

// LDS: 64 KiB table, each lane a random dword (K = 64) or 64/K lanes per 128 B.
__global__ void __launch_bounds__(1024) k_lds(uint32_t k, uint32_t *out) {
    extern __shared__ uint32_t lds[];
    for (uint32_t i = threadIdx.x; i < 16384; i += blockDim.x) lds[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t grp = lane / (64u / k), sub = lane % (64u / k);
    uint32_t acc = 0, seed = wave * 7919u;
    for (int i = 0; i < ITERS; i += 4) {
        uint32_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t line = mix(seed + (i + j) * 131u + grp * 977u) & 511u;
            v[j] = lds[line * 32u + sub % 32u];
        }
        acc += v[0] ^ v[1] ^ v[2] ^ v[3];
        seed ^= acc & 1u;
    }
    if (acc == 0x12345678u) out[wave] = acc;
}

int main() {
    int dev = 0, cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const size_t max_bytes = size_t(64) << 20;
    uint32_t *tab = nullptr, *out = nullptr;
    CK(hipMalloc(&tab, max_bytes));
    CK(hipMemset(tab, 1, max_bytes));
    const uint32_t blocks = uint32_t(cus) * 2, threads = 1024, waves = blocks * threads / 64;
    CK(hipMalloc(&out, waves * 4));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto timed = [&](auto launch) -> double {
        launch();
        if (hipDeviceSynchronize() != hipSuccess) return -1.0;
        (void)hipEventRecord(a);
        for (int r = 0; r < 10; ++r) launch();
        (void)hipEventRecord(b);
        if (hipEventSynchronize(b) != hipSuccess) return -1.0;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        return double(ms) / 10.0;
    };
    std::printf("{\"cus\": %d, \"waves\": %u, \"iters\": %d, \"results\": [\n", cus, waves, ITERS);
    bool first = true;
    for (size_t bytes : {size_t(256) << 10, size_t(2) << 20, size_t(16) << 20, size_t(64) << 20})
        for (int w : {1, 4})
            for (uint32_t k : {1u, 2u, 4u, 8u, 16u, 32u, 64u}) {
                const uint32_t lines = uint32_t(bytes / 128);
                double ms = -1;
                if (w == 1) ms = timed([&] { hipLaunchKernelGGL(k_gather<1>, blocks, threads, 0, 0, tab, lines, k, out); return 0; });
                else ms = timed([&] { hipLaunchKernelGGL(k_gather<4>, blocks, threads, 0, 0, tab, lines, k, out); return 0; });
                const double ns = ms * 1e6 * cus / (double(waves) * ITERS);
                std::printf("%s {\"table_bytes\": %zu, \"bytes_per_lane\": %d, \"lines_per_instr\": %u, \"ms\": %.4f, \"ns_per_instr_per_cu\": %.3f}",
                            first ? "" : ",\n", bytes, 4 * w, k, ms, ns);
                first = false;
            }
    for (size_t bytes : {size_t(2) << 20, size_t(5) << 20, size_t(16) << 20})
        for (int pair : {0, 1}) {
            const uint32_t ents = uint32_t(bytes / 24);
            double ms = pair ? timed([&] { hipLaunchKernelGGL(k_ent24<1>, blocks, threads, 0, 0, tab, ents, out); return 0; })
                             : timed([&] { hipLaunchKernelGGL(k_ent24<0>, blocks, threads, 0, 0, tab, ents, out); return 0; });
            // entries loaded: PAIR 0: 64 per instruction step, PAIR 1: 32
            const double per64 = ms * 1e6 * cus / (double(waves) * ITERS * (pair ? 0.5 : 1.0));
            std::printf(",\n {\"entries24\": true, \"table_bytes\": %zu, \"pair\": %d, \"ms\": %.4f, \"ns_per_64_entries_per_cu\": %.3f}",
                        bytes, pair, ms, per64);
        }
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(k_lds), hipFuncAttributeMaxDynamicSharedMemorySize, 65536));
    for (uint32_t k : {1u, 8u, 64u}) {
        double ms = timed([&] { hipLaunchKernelGGL(k_lds, blocks, threads, 65536, 0, k, out); return 0; });
        const double ns = ms * 1e6 * cus / (double(waves) * ITERS);
        std::printf(",\n {\"lds\": true, \"lines_per_instr\": %u, \"ms\": %.4f, \"ns_per_instr_per_cu\": %.3f}", k, ms, ns);
    }
    std::printf("\n]}\n");
    return 0;
}
