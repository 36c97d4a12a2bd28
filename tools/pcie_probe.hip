// pcie_probe — how long does one wave take to read N bytes of pinned host
// memory over PCIe, by allocation kind, cache policy of the load and number
// of waves reading at once?  Experiment for the burst consumer's mailbox poll
// (DESIGN.md §4.7): the poll round trip, not the classification, bounds a
// 32-packet burst call.  Every kernel is bounded (iters reads, then exit); the
// host never changes the data, so a policy that caches shows up as a fast
// repeat read (stale data: unusable for a mailbox).
// usage: pcie_probe  -> one JSON line per (memory, policy, bytes, waves)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x)                                                                  \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));  \
            return 1;                                                             \
        }                                                                         \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Each workgroup (one wave) reads `loads` x 1 KiB (16 B per lane) from its own
// 4 KiB region, `iters` times, waiting for every read before the next pass;
// out[wg] = wall-clock ticks (100 MHz) of all passes.
template <int AUX>
__global__ void k_read(const uint8_t *base, uint32_t loads, uint32_t lanes, uint32_t iters, uint64_t *out,
                       uint32_t *sink) {
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base) + size_t(blockIdx.x) * 4096, 0, 4096, 0x00020000);
    uint32_t acc = 0;
    const uint64_t t0 = wall_clock64();
    for (uint32_t it = 0; it < iters; ++it) {
        u32x4 v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (q < int(loads) && lane < lanes)
                v[q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, int(q * 1024 + lane * 16), 0, AUX));
            else
                v[q] = u32x4{0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) acc += v[q].x ^ v[q].w;
        acc = __builtin_amdgcn_readfirstlane(acc);  // forces the wait for every read of this pass
    }
    const uint64_t t1 = wall_clock64();
    if (lane == 0) out[blockIdx.x] = t1 - t0;
    if (acc == 0x12345678u) sink[0] = acc;
}

template <int AUX>
static int run(const char *mem, const char *pol, uint8_t *h, uint64_t *d_out, uint32_t *sink) {
    const uint32_t iters = 2000;
    for (uint32_t loads : {1u, 2u, 4u}) {
        for (uint32_t lanes : {4u, 64u}) {
            if (lanes == 4 && loads != 1) continue;
            for (uint32_t waves : {1u, 16u, 32u, 64u}) {
                hipLaunchKernelGGL(k_read<AUX>, dim3(waves), dim3(64), 0, 0, h, loads, lanes, iters, d_out, sink);
                CHECK(hipDeviceSynchronize());
                std::vector<uint64_t> t(waves);
                CHECK(hipMemcpy(t.data(), d_out, waves * 8, hipMemcpyDeviceToHost));
                double mean = 0;
                for (uint64_t x : t) mean += double(x);
                mean /= waves;
                const double us = mean / iters / 100.0;  // 100 MHz ticks -> us per pass
                const double bytes = double(loads) * lanes * 16;
                std::printf("{\"mem\": \"%s\", \"policy\": \"%s\", \"bytes\": %.0f, \"waves\": %u, \"us_per_read\": %.3f, "
                            "\"GBps_total\": %.2f}\n",
                            mem, pol, bytes, waves, us, bytes * waves / us / 1e3);
                std::fflush(stdout);
            }
        }
    }
    return 0;
}

int main() {
    uint64_t *d_out;
    uint32_t *sink;
    CHECK(hipMalloc(&d_out, 64 * 8));
    CHECK(hipMalloc(&sink, 4));
    struct Kind {
        const char *name;
        unsigned flags;
    } kinds[] = {{"coherent", hipHostMallocDefault}, {"noncoherent", hipHostMallocNonCoherent},
                 {"writecombined", hipHostMallocWriteCombined}};
    for (const Kind &k : kinds) {
        uint8_t *h = nullptr;
        if (hipHostMalloc(&h, 64 * 4096, k.flags) != hipSuccess) {
            std::printf("{\"mem\": \"%s\", \"error\": \"alloc\"}\n", k.name);
            continue;
        }
        for (int i = 0; i < 64 * 4096; ++i) h[i] = uint8_t(i * 7);
        if (run<17>(k.name, "sc0sc1", h, d_out, sink)) return 1;
        if (run<16>(k.name, "sc1", h, d_out, sink)) return 1;
        if (run<1>(k.name, "sc0", h, d_out, sink)) return 1;
        if (run<3>(k.name, "sc0nt", h, d_out, sink)) return 1;
        if (run<0>(k.name, "default", h, d_out, sink)) return 1;
        CHECK(hipHostFree(h));
    }
    return 0;
}
