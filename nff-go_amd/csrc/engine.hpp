// engine.hpp — engine object behind the nffacl_engine handle (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>

#include "compile.hpp"

namespace nffacl {

void set_last_error(const std::string &s);
const char *last_error();

// One compiled table resident in HBM.
struct DevTable {
    uint32_t *d_blob = nullptr;
    size_t bytes = 0;
    CompiledTable meta;
    ~DevTable();
};

int upload_table(int device, const nffacl_rules &rules, int algo, DevTable *&out);

}  // namespace nffacl

struct nffacl_engine {
    int device = 0;
    int algo_req = NFFACL_ALGO_AUTO;
    int num_cus = 256;
    // Active table (read by every launch) and the table it replaced, kept
    // alive until the next swap has drained the device.
    std::mutex table_mu;
    nffacl::DevTable *active = nullptr;
    nffacl::DevTable *retired = nullptr;
    // Host-inclusive pipeline state (nffacl_classify_host), created lazily.
    std::mutex host_mu;
    size_t chunk = 0;
    uint8_t *h_stage[2] = {nullptr, nullptr};
    uint32_t *h_port[2] = {nullptr, nullptr};
    uint8_t *d_slots[2] = {nullptr, nullptr};
    uint32_t *d_port[2] = {nullptr, nullptr};
    hipStream_t streams[2] = {nullptr, nullptr};
    hipEvent_t done[2] = {nullptr, nullptr};
    uint32_t staged_stride = 0;
};

namespace nffacl {
// The table launches issued now must use (swap_rules may replace it later).
inline DevTable *acquire_table(nffacl_engine *eng) {
    std::lock_guard<std::mutex> g(eng->table_mu);
    return eng->active;
}
int prepare_kernels();
int launch_slots(nffacl_engine *eng, const DevTable *t, const uint8_t *d_slots, uint32_t stride,
                 uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream, uint32_t flags = 0);
int launch_frames(nffacl_engine *eng, const DevTable *t, const uint8_t *d_frames,
                  const uint64_t *d_desc, uint64_t n, uint32_t *d_port, uint64_t *d_permit,
                  hipStream_t stream, uint32_t flags = 0);
}  // namespace nffacl
