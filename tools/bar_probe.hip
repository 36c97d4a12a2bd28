// bar_probe — can the host write device memory directly (large BAR), and how
// fast does a GPU poll of local memory see a host write, compared with a GPU
// poll of pinned host memory?  Experiment for the scalar-call consumer
// (DESIGN.md §4.7): a request crossing PCIe as a posted host write instead of
// a GPU read round trip.
//
// Every host access to device memory runs in a forked child first (a host
// fault then only ends the child).  The GPU kernel is bounded: it polls at
// most `iters` times and exits.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));      \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

// Ping-pong: the host writes seq to `in`, the kernel waits for it and writes
// seq to `out` (pinned host memory); `rounds` round trips, each bounded.
__global__ void k_pong(const uint32_t *in, uint32_t *out, uint32_t rounds, uint64_t max_ticks) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = wall_clock64();
    for (uint32_t r = 1; r <= rounds; ++r) {
        while (__hip_atomic_load(in, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != r) {
            if (wall_clock64() - t0 > max_ticks) return;  // bounded: 2 s at most
        }
        __hip_atomic_store(out, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double pingpong(volatile uint32_t *h_in, const uint32_t *d_in, volatile uint32_t *h_out, uint32_t *d_out,
                       uint32_t rounds) {
    *h_in = 0;
    *h_out = 0;
    hipLaunchKernelGGL(k_pong, dim3(1), dim3(64), 0, 0, d_in, d_out, rounds, 200000000ull);  // 2 s at 100 MHz
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    std::vector<double> lat;
    for (uint32_t r = 1; r <= rounds; ++r) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(const_cast<uint32_t *>(h_in), r, __ATOMIC_RELEASE);
        const auto limit = t0 + std::chrono::milliseconds(100);
        while (__atomic_load_n(const_cast<uint32_t *>(h_out), __ATOMIC_ACQUIRE) != r)
            if (std::chrono::steady_clock::now() > limit) break;
        lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    (void)hipDeviceSynchronize();
    std::sort(lat.begin(), lat.end());
    return lat[lat.size() / 2];
}

int main() {
    CHECK(hipSetDevice(0));
    uint32_t *h_pin = nullptr, *d_pin = nullptr;
    CHECK(hipHostMalloc(reinterpret_cast<void **>(&h_pin), 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&d_pin), h_pin, 0));
    // 1. baseline: both words in pinned host memory (GPU polls over PCIe)
    const double host_poll = pingpong(h_pin, d_pin, h_pin + 16, d_pin + 16, 2000);
    // 2. device fine-grained memory written by the host
    uint32_t *d_fg = nullptr;
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void **>(&d_fg), 4096, hipDeviceMallocFinegrained);
    hipPointerAttribute_t at;
    std::memset(&at, 0, sizeof at);
    int host_ok = 0;
    if (e == hipSuccess) {
        (void)hipPointerGetAttributes(&at, d_fg);
        const pid_t pid = fork();
        if (pid == 0) {  // child: touch it from the host
            volatile uint32_t *p = d_fg;
            p[1] = 0x5a5a5a5a;
            _exit(p[1] == 0x5a5a5a5a ? 0 : 2);
        }
        int status = 0;
        waitpid(pid, &status, 0);
        host_ok = WIFEXITED(status) && WEXITSTATUS(status) == 0;
    }
    double dev_poll = -1;
    if (host_ok) dev_poll = pingpong(d_fg, d_fg, h_pin + 32, d_pin + 32, 2000);
    std::printf("{\"host_pinned_poll_rt_us_p50\": %.2f, \"finegrained_alloc\": \"%s\", \"attr_type\": %d, "
                "\"attr_hostptr\": %d, \"host_can_write_vram\": %d, \"vram_poll_rt_us_p50\": %.2f}\n",
                host_poll, hipGetErrorString(e), int(at.type), at.hostPointer != nullptr, host_ok, dev_poll);
    return 0;
}
