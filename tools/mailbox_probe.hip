// mailbox_probe — the burst mailbox round trip in isolation:
// one host thread writes a request (`body` bytes of 16-byte chunks, then a
// 32-byte header carrying the tag) into pinned host memory and spins on the
// response word; one GPU wave polls, reads the request, answers.  Variants:
//   full: the wave reads the whole mailbox every pass (round-3/4 consumer);
//   hdr:  the wave polls the header only and reads the body once it changed;
// host stores plain or streaming (nt).  Reports host-side round trip p50/p99
// and the wave's mean header-poll and body-read times.  Every kernel is
// bounded (it leaves after `rounds` requests or 2 s).
// usage: mailbox_probe [cpu]  -> one JSON line per variant
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

__device__ __forceinline__ u32x4 ld16(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(off), 0, 17));
}

// stats: [0] polls, [1] poll ticks, [2] body reads, [3] body ticks.
// PIPE (full polls only): the next poll is issued before the current one's
// request is answered, as the service's consumer does.
// Service-like extras: `ctrl` != null: one system-scope 8-byte load of it per
// pass (the consumer's stop word); `resp_lanes` lanes answer (one 8-byte
// system-scope store each, as 32 packets); `work` wall-clock ticks spent
// between reading a request and answering it (the classification).
template <bool HDR, bool PIPE>
__global__ void k_box(const uint8_t *box, uint32_t body_loads, uint64_t *resp, uint32_t rounds, uint64_t *stats,
                      const uint64_t *ctrl, uint32_t resp_lanes, uint32_t work) {
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(box), 0, 4096, 0x00020000);
    const uint64_t t0 = wall_clock64();
    uint32_t done = 0;
    uint64_t np = 0, pt = 0, nb = 0, bt = 0;
    u32x4 nx[4] = {};
    uint64_t ta = 0;
    auto issue = [&]() {
        ta = wall_clock64();
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) nx[j] = u32x4{0, 0, 0, 0};
        if (HDR) {
            if (lane < 2) nx[0] = ld16(rs, 16u * lane);
        } else {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (j < body_loads) nx[j] = ld16(rs, 1024u * j + 16u * lane);
        }
    };
    issue();
    while (done < rounds && wall_clock64() - t0 < 200000000ull) {
        u32x4 v[4];
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) v[j] = nx[j];
        const uint64_t a = ta;
        uint64_t cw = 0;
        if (ctrl && lane == 0) cw = __hip_atomic_load(ctrl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t tag = __builtin_amdgcn_readlane(v[0].w, 0);
        const uint32_t last = __builtin_amdgcn_readlane(v[body_loads - 1].w, 63);
        if (__builtin_amdgcn_readlane(static_cast<uint32_t>(cw), 0) == 0xDEADBEEFu) break;
        __builtin_amdgcn_s_waitcnt(0);  // (the clock read after the data, not hoisted above the wait)
        const uint64_t b = wall_clock64();
        ++np;
        pt += b - a;
        if (PIPE) issue();
        if (tag == done) {
            if (!PIPE) issue();
            continue;
        }
        uint32_t lt = last;
        if (HDR) {
#pragma unroll
            for (uint32_t j = 0; j < 4; ++j)
                if (j < body_loads) v[j] = ld16(rs, 1024u * j + 16u * lane);
            lt = __builtin_amdgcn_readlane(v[body_loads - 1].w, 63);
            __builtin_amdgcn_s_waitcnt(0);
            const uint64_t c = wall_clock64();
            ++nb;
            bt += c - b;
        }
        // the last chunk carries the tag too: torn reads retry
        if (lt == tag) {
            if (work) {
                const uint64_t w0 = wall_clock64();
                while (wall_clock64() - w0 < work) {
                }
            }
            done = tag;
            if (lane < resp_lanes)
                __hip_atomic_store(resp + lane, uint64_t(tag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (!PIPE) issue();
    }
    if (lane == 0) {
        stats[0] = np;
        stats[1] = pt;
        stats[2] = nb;
        stats[3] = bt;
    }
}

// Round trip of one 32-byte poll of unchanged host memory, `iters` in a row.
__global__ void k_rt(const uint8_t *box, uint32_t iters, uint64_t *stats) {
    const uint32_t lane = threadIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(box), 0, 4096, 0x00020000);
    uint32_t acc = 0;
    const uint64_t a = wall_clock64();
    for (uint32_t i = 0; i < iters; ++i) {
        u32x4 v = {};
        if (lane < 2) v = ld16(rs, 16u * lane + (acc & 16u));
        acc += __builtin_amdgcn_readlane(v.w, 0) + 1u;
        __builtin_amdgcn_s_waitcnt(0);
    }
    const uint64_t b = wall_clock64();
    if (lane == 0) {
        stats[0] = b - a;
        stats[1] = acc;
    }
}

static void put(__m128i *d, __m128i v, bool nt) {
    if (nt) _mm_stream_si128(d, v);
    else _mm_store_si128(d, v);
}

int main(int argc, char **argv) {
    if (argc > 1) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(std::atoi(argv[1]), &set);
        (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
    }
    uint8_t *box;
    uint64_t *resp, *stats;
    CHECK(hipHostMalloc(&box, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostMalloc(&resp, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipMalloc(&stats, 64));
    const uint32_t rounds = 4000;
    {
        struct K { const char *name; unsigned flags; } kinds[] = {
            {"mapped_coherent", hipHostMallocMapped | hipHostMallocCoherent}, {"default", hipHostMallocDefault},
            {"mapped_noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent}};
        for (const K &k : kinds) {
            uint8_t *b2;
            CHECK(hipHostMalloc(&b2, 4096, k.flags));
            std::memset(b2, 1, 4096);
            hipLaunchKernelGGL(k_rt, dim3(1), dim3(64), 0, 0, b2, 2000u, stats);
            CHECK(hipDeviceSynchronize());
            uint64_t st[2];
            CHECK(hipMemcpy(st, stats, 16, hipMemcpyDeviceToHost));
            std::printf("{\"static_poll\": \"%s\", \"rt_us\": %.3f}\n", k.name, double(st[0]) / 2000 / 100.0);
            CHECK(hipHostFree(b2));
        }
    }
    uint64_t *ctrl;
    CHECK(hipHostMalloc(&ctrl, 64, hipHostMallocMapped | hipHostMallocCoherent));
    *ctrl = 0;
    struct V { const char *name; bool use_ctrl; uint32_t lanes; uint32_t work; } vs[] = {
        {"plain", false, 1, 0}, {"ctrl", true, 1, 0}, {"resp32", false, 32, 0}, {"work1.25us", false, 1, 125},
        {"service_like", true, 32, 125}};
    for (const V &v : vs) {
        const uint32_t loads = 4;
        std::memset(box, 0, 4096);
        std::memset(resp, 0, 4096);
        *resp = 0;
        hipLaunchKernelGGL((k_box<false, false>), dim3(1), dim3(64), 0, 0, box, loads, resp, rounds, stats,
                           v.use_ctrl ? ctrl : nullptr, v.lanes, v.work);
        std::vector<double> lat;
        for (uint32_t tag = 1; tag <= rounds; ++tag) {
            const auto t0 = std::chrono::steady_clock::now();
            __m128i *d = reinterpret_cast<__m128i *>(box);
            for (uint32_t c = loads * 64; c-- > 2;) put(d + c, _mm_set_epi32(int(tag), 1, 2, 3), false);
            put(d + 1, _mm_set_epi32(int(tag), 0, 0, 32), false);
            put(d, _mm_set_epi32(int(tag), 7, 8, 9), false);
            const auto limit = t0 + std::chrono::milliseconds(50);
            bool ok = true;
            const uint32_t want = v.lanes > 1 ? 31 : 0;
            while (__atomic_load_n(resp + want, __ATOMIC_ACQUIRE) != tag) {
                _mm_pause();
                if (std::chrono::steady_clock::now() > limit) { ok = false; break; }
            }
            if (!ok) break;
            lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        *ctrl = 0xDEADBEEFull;
        CHECK(hipDeviceSynchronize());
        *ctrl = 0;
        uint64_t st[4];
        CHECK(hipMemcpy(st, stats, 32, hipMemcpyDeviceToHost));
        std::sort(lat.begin(), lat.end());
        auto pct = [&](double p) { return lat.empty() ? 0.0 : lat[std::min(lat.size() - 1, size_t(p * lat.size()))]; };
        std::printf("{\"variant\": \"%s\", \"answered\": %zu, \"p50_us\": %.2f, \"p99_us\": %.2f, \"poll_us\": %.3f, "
                    "\"polls_per_req\": %.2f}\n",
                    v.name, lat.size(), pct(0.5), pct(0.99), st[0] ? double(st[1]) / st[0] / 100.0 : 0.0,
                    lat.empty() ? 0.0 : double(st[0]) / lat.size());
        std::fflush(stdout);
    }
    return 0;
}
