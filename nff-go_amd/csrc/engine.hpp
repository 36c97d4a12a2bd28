// engine.hpp — engine object behind the nffacl_engine handle (internal).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "compile.hpp"
#include "tables.hpp"

namespace nffacl {

void set_last_error(const std::string &s);
const char *last_error();

// One compiled table resident in HBM (lifetime: tables.hpp).  The blob is
// followed by the scalar-call consumer's descriptor (service.hpp SvcDesc).
struct DevTable : DeviceBlob {
    CompiledTable meta;
    uint32_t gen = 0;                  // upload epoch: process-unique, increasing (service.hip)
    uint32_t svc_kind = 0;             // SvcKind of the layout
    const uint32_t *d_desc = nullptr;  // device address of the SvcDesc
};
using TablePtr = std::shared_ptr<DevTable>;

// Launch-shape knobs, read from the environment ONCE at engine creation
// (tools/ab_env.py experiments; unset in production) and validated there —
// never on the launch path.
struct Tune {
    int coal = 4;    // NFFACL_TUNE_COAL: 64-byte slot load mode 0..5 (engine.hip)
    bool coal_set = false;  // the mode was set explicitly (else: 5 for kTabFlatLds4U walks)
    int block = 0;   // NFFACL_TUNE_BLOCK: threads per workgroup (0 = kernel default)
    int per_cu = 0;  // NFFACL_TUNE_PER_CU: workgroups per CU (0 = kernel default)
    int rounds = 0;  // NFFACL_TUNE_ROUNDS: flat walks, loads in flight (0 = compiled, 2 or 4)
    int lds = 1;     // NFFACL_TUNE_LDS: 0 keeps INDEXED tables in global memory
    int dyn = 1;     // NFFACL_TUNE_DYN: batch kernels pull their batches (engine.hip BatchSource):
                     // 1 the flat-LDS slot walks, 2 every indexed batch kernel, 0 none (grid stride)
    // pull sizes: at most dyn_gmax batches and about a dyn_pulls-th of a
    // wave's share; near a head's end (head's remaining batches) /
    // (waves x dyn_tail / 16), at least dyn_gmin
    int dyn_gmax = 16, dyn_gmin = 12, dyn_pulls = 4, dyn_tail = 2;
    int pipe = 1;    // NFFACL_TUNE_PIPE: 1 flat-LDS positional tables with many candidates per packet
                     // (flat_uncond: C5) take the pipelined walk (classify_flat_pipe); 2 all of them; 0 none
    // nffacl_classify_host (capi.cpp): pinned input read by the kernel over
    // PCIe (0) or DMA'd to HBM first (1); buffers = streams in flight (2..4);
    // packets per chunk, log2
    int host_dma = 0;      // NFFACL_TUNE_HOST_DMA
    int host_bufs = 3;     // NFFACL_TUNE_HOST_BUFS
    int host_chunk = 20;   // NFFACL_TUNE_HOST_CHUNK (log2, 12..24)
    CompileOptions copt;  // NFFACL_TUNE_FLAT / _DIR_KB / _DIR16 (table layout)
    // false (+ `err`) if a set variable is out of range
    static bool from_env(Tune &t, std::string &err);
};

// Pull heads of the batch kernels (engine.hip BatchSource): eight heads and a
// finish counter, a 128-byte line each, per stream an engine launches on.
constexpr uint32_t kDynHeadStride = 32;
constexpr uint32_t kDynBlockWords = 9 * kDynHeadStride;

int upload_table(nffacl_engine *eng, const nffacl_rules &rules, TablePtr &out);
// An engine without a table (launch shape of `hip_device` only): the device
// batcher's, whose batches take their rule sets' own tables (capi.cpp).
int engine_shell(int hip_device, nffacl_engine **out);
// Compile `rules` with `algo` / `copt`, upload blob + service descriptor
// through `home` (whose device is current), fill `t`.
int compile_upload(const nffacl_rules &rules, int algo, const CompileOptions &copt, TableHome &home, DevTable &t);
// The device image of a compiled table (blob + service descriptor) in
// `words`, its metadata in `t`; table_resident() completes `t` once its
// d_blob holds the words (the group's RCCL broadcast, group.cpp).
int compile_words(const nffacl_rules &rules, int algo, const CompileOptions &copt, DevTable &t,
                  std::vector<uint32_t> &words);
void table_resident(DevTable &t);
// Generation of the latest completed table upload.
uint32_t table_epoch();

}  // namespace nffacl

struct nffacl_engine {
    int device = 0;
    int algo_req = NFFACL_ALGO_AUTO;
    int num_cus = 256;
    nffacl::Tune tune;
    // Table uploads + stream-ordered frees of retired tables.  Declared
    // before `active` so that it is destroyed after it.
    nffacl::TableHome home;
    // The table launches issued now use (swap_rules replaces it; holders of
    // the previous one keep it alive, tables.hpp).
    std::mutex table_mu;
    nffacl::TablePtr active;
    // Host-inclusive pipeline state (nffacl_classify_host), created lazily.
    std::mutex host_mu;
    static constexpr int kHostBufs = 4;
    size_t chunk = 0;
    int nbufs = 0;
    uint8_t *h_stage[kHostBufs] = {};    // pinned input staging (pageable callers)
    uint32_t *h_port[kHostBufs] = {};    // mapped pinned verdict staging
    uint32_t *d_hport[kHostBufs] = {};   // their device aliases (the kernels write there)
    uint8_t *d_slots[kHostBufs] = {};    // HBM input chunks (DMA forms)
    hipStream_t streams[kHostBufs] = {};
    hipEvent_t done[kHostBufs] = {};
    uint32_t staged_stride = 0;
    // BatchSource heads: block i serves dyn_stream[i] (launches on one stream
    // are ordered, and each launch leaves its block zeroed for the next);
    // streams beyond kDynStreams launch with the fixed grid stride
    static constexpr int kDynStreams = 64;
    std::mutex dyn_mu;
    uint32_t *d_dyn = nullptr;
    hipStream_t dyn_stream[kDynStreams] = {};
    int dyn_used = 0;
};

namespace nffacl {
// The table launches issued now must use; the caller holds it while it
// enqueues work (swap_rules may replace it meanwhile).
inline TablePtr acquire_table(nffacl_engine *eng) {
    std::lock_guard<std::mutex> g(eng->table_mu);
    return eng->active;
}
int prepare_kernels();
// nffacl_engine_kernel_info: the slot kernel of the active table.
int slots_kernel_info(nffacl_engine *eng, nffacl_kernel_info *out);
// Both record the launch on `t` (DeviceBlob::note_use) so that a retired
// table outlives the work enqueued with it.
int launch_slots(nffacl_engine *eng, DevTable *t, const uint8_t *d_slots, uint32_t stride,
                 uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream, uint32_t flags = 0);
int launch_frames(nffacl_engine *eng, DevTable *t, const uint8_t *d_frames,
                  const uint64_t *d_desc, uint64_t n, uint32_t *d_port, uint64_t *d_permit,
                  hipStream_t stream, uint32_t flags = 0);
}  // namespace nffacl
