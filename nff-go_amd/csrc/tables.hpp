// tables.hpp — lifetime of device rule tables under concurrent swap (internal).
//
// The reference hot-swaps rules by storing a new *L3Rules pointer while
// flow-function clones keep classifying with the old one (user code,
// examples/tutorial/step08.go:33-44); Go's GC frees the old table once no
// goroutine holds it.  Here a table is held by std::shared_ptr: every launch,
// host pipeline call and batcher launch copies the engine's active pointer
// under the engine lock and holds it while it enqueues work.  Device work
// outlives the host reference, so every launch also records a completion
// event on its stream (one reusable event per stream per table: work on a
// stream completes in order, so the latest record covers all earlier ones).
// When the last host reference drops, the table's device blob is retired
// without blocking anyone: the engine's private stream waits on those events
// and frees the blob stream-ordered (hipFreeAsync) behind them.  No
// hipDeviceSynchronize, no wait on unrelated streams.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace nffacl {

void set_last_error(const std::string &s);

// Per engine: the stream that uploads tables and frees retired ones, and the
// events of retired tables until that stream has passed them.
struct TableHome {
    int device = 0;
    hipStream_t stream = nullptr;  // non-blocking: never orders against user streams
    // stream-ordered allocator available (hipMallocAsync); cleared by the
    // first upload it refuses, read by whichever thread retires a table
    std::atomic<bool> pools{false};
    std::mutex mu;
    struct Grave {
        std::vector<hipEvent_t> evs;  // the retired table's per-stream completion events
        hipEvent_t fence = nullptr;   // recorded on `stream` after the waits (and the free)
        void *blob = nullptr;         // !pools: freed with hipFree once `fence` has fired
    };
    std::vector<Grave> graves;

    hipError_t init(int dev);
    // Release graves whose fence has fired; wait for all of them if `all`.
    void reap(bool all);
    // Engine teardown: wait for the private stream, release everything.
    void shutdown();
    ~TableHome() { shutdown(); }
};

// Device blob of one compiled table.  Derived types add the host metadata.
struct DeviceBlob {
    uint32_t *d_blob = nullptr;
    size_t bytes = 0;
    TableHome *home = nullptr;

    // Record that work reading this blob was just enqueued on `s`.
    hipError_t note_use(hipStream_t s);
    // Allocate + upload `words` on home->stream (synchronous w.r.t. that
    // stream only); the blob is usable by any stream when this returns.
    hipError_t upload(TableHome *h, const uint32_t *words, size_t n_words);
    // Allocate only (the words arrive by other means: group.cpp's broadcast).
    hipError_t alloc(TableHome *h, size_t n_words);

    DeviceBlob() = default;
    DeviceBlob(const DeviceBlob &) = delete;
    DeviceBlob &operator=(const DeviceBlob &) = delete;
    virtual ~DeviceBlob();  // retire: stream-ordered free behind every recorded use

  private:
    std::mutex use_mu_;
    std::vector<std::pair<hipStream_t, hipEvent_t>> uses_;
};

}  // namespace nffacl
