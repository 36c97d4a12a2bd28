// batcher.hpp — multi-producer burst aggregator behind nffacl_batcher (internal).
//
// The reference classifies inside each flow-function clone, one burst of <= 32
// packets at a time (segmentProcess, flow/flow.go:1487-1520, calling the
// VectorSeparateFunction of flow.go:131).  A GPU launch per burst is latency
// bound, so the batcher lets every clone (thread) submit its burst into a
// shared pinned slot ring; one launcher thread ships the open batch as soon as
// fewer than two batches are on the GPU (adaptive batching: it grows while the
// GPU is busy, up to max_batch; batcher.cpp), and each clone sleeps only until
// its own batch's verdicts are back.
//
// Buffers: `nbuf` batch buffers, each = mapped pinned slots + ports on the host
// (the kernel reads the slots and writes the verdicts over PCIe directly:
// one launch per batch, no copies), a stream and an event.  States cycle
//   FREE -> OPEN (accepting bursts) -> SEALED -> LAUNCHED -> DONE -> FREE
// (DONE -> FREE once every burst of the batch has collected its verdicts).
// A batch classifies against ONE table: the engine's active table at launch,
// or the table of the rule set its bursts were submitted with
// (nffacl_batcher_submit_rules) — a burst for another table seals the open
// batch and starts the next.  Each batch carries its own status: a failed
// launch fails that batch's bursts only.
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "engine.hpp"
#include "nffacl.h"

namespace nffacl {

struct BatchBuf {
    enum State { FREE, OPEN, SEALED, LAUNCHED, DONE };
    State state = FREE;
    // batch sequence number (written under the batcher mutex when the buffer
    // opens; waiters read it without the lock to reject stale tickets)
    std::atomic<uint64_t> seq{0};
    uint32_t count = 0;     // packets reserved
    uint32_t bursts = 0;    // bursts reserved (ticket burst numbers 0..bursts-1)
    // the rule set's table every burst of this batch was submitted with, or
    // nullptr: the engine's active table at launch (kept alive by the
    // submitters, who wait for the batch before they may free their rules)
    DevTable *table = nullptr;
    std::atomic<uint32_t> readers{0};  // bursts that have not collected their verdicts yet
    std::atomic<uint32_t> written{0};  // packets whose bytes are in h_slots
    std::atomic<uint64_t> done_seq{0}; // == seq once the verdicts are in h_port (or the batch failed)
    std::atomic<int> status{NFFACL_OK};  // this batch's outcome, published before done_seq
    // bumped after done_seq: waiters sleep on it (futex; one wake releases
    // all of them at once, no mutex to re-take)
    std::atomic<uint32_t> gen{0};
    // per burst number: the seq of the batch whose burst collected it (a
    // second wait on the same ticket is rejected instead of freeing the
    // buffer twice)
    std::unique_ptr<std::atomic<uint64_t>[]> claimed;
    // per burst number: the submitting thread's outstanding-ticket counter
    // (nffacl_batcher::owners), decremented by whichever thread collects it
    std::unique_ptr<std::atomic<int64_t> *[]> owner;
    std::chrono::steady_clock::time_point opened;
    uint8_t *h_slots = nullptr;   // mapped pinned host memory
    uint32_t *h_port = nullptr;
    uint8_t *d_slots = nullptr;   // device aliases of h_slots / h_port
    uint32_t *d_port = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
};

}  // namespace nffacl

struct nffacl_batcher {
    nffacl_engine *eng = nullptr;     // launch shape + (engine batchers) the active table
    bool own_eng = false;             // device batcher: a table-less engine shell of its own
    uint32_t stride = 64;
    uint32_t max_batch = 0;
    std::chrono::microseconds max_delay{100};  // longest wait behind a full pipeline
    // longest back-pressure wait of a submit before NFFACL_ERR_TIMEOUT
    // (NFFACL_TUNE_BATCH_SUBMIT_MS, tests)
    std::chrono::milliseconds submit_bound{1000};
    // the same for a caller holding no uncollected ticket, who waits on other
    // threads' batches (NFFACL_TUNE_BATCH_FOREIGN_MS)
    std::chrono::milliseconds foreign_bound{30000};
    uint64_t id = 0;  // process-unique (this thread's own tickets, batcher.cpp)
    // one outstanding-ticket counter per submitting thread, owned here (a
    // ticket may be collected on another thread, or after its submitter
    // exited); under `mu`
    std::vector<std::unique_ptr<std::atomic<int64_t>>> owners;
    uint32_t nbuf = 0;
    std::unique_ptr<nffacl::BatchBuf[]> bufs;

    std::mutex mu;
    std::condition_variable cv_work;  // launcher: a batch sealed / opened / a buffer freed
    std::condition_variable cv_free;  // producers: a buffer became FREE
    uint32_t open_idx = 0;            // buffer producers append to
    uint32_t launch_idx = 0;          // next buffer the launcher ships
    uint64_t next_seq = 1;
    bool stop = false;
    bool launcher_done = false;

    std::deque<uint32_t> inflight;    // launched buffers, FIFO
    uint32_t inflight_n = 0;          // batches launched (or launching) and not completed
    uint32_t busy = 0;                // buffers not FREE
    // Waiters spin (no syscalls) only while fewer than spin_limit of them do:
    // past the host's CPU share, spinning submitters would starve the
    // launcher and completer threads (batcher.cpp)
    std::atomic<uint32_t> spinners{0};
    uint32_t spin_limit = 1;
    // NFFACL_TUNE_BATCH_FAIL_AT (tests): the launch with this number (1-based)
    // fails as a HIP error would; NFFACL_TUNE_BATCH_HOLD=1 (tests): nothing
    // ships before flush (a batch that never completes on its own)
    uint64_t fail_at = 0;
    bool hold = false;
    uint64_t launch_no = 0;
    std::condition_variable cv_inflight;
    std::thread launcher, completer;

    // stats
    uint64_t batches = 0, packets = 0, bursts = 0, timeouts = 0;  // timeouts: shipped before full
    uint64_t failed = 0;                                          // batches whose launch failed
};
