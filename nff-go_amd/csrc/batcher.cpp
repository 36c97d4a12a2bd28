// batcher.cpp — nffacl_batcher: multi-producer burst aggregation onto the GPU
// (see batcher.hpp).  One launcher thread seals and ships batches in ring
// order; one completer thread waits on their events in launch order and
// publishes each batch's sequence number, on which the bursts' submitters spin.
//
// Launch policy (adaptive batching): a batch ships as soon as it holds a burst,
// fewer than kEagerInflight batches are on the GPU and a buffer stays free
// behind it, so an idle GPU costs a burst one launch round trip, while a busy
// one lets the open batch grow (up to max_batch) until a batch completes.  A
// batch whose first burst has waited max_delay_us ships in any case: no
// number of buffers and no wait order of the submitters' tickets can hold it
// back (buffers whose tickets are not collected yet stay busy).
// The reference's clones submit synchronously (segmentProcess waits for its
// separator's answers, flow/flow.go:1487-1520), so the open batch collects
// exactly the bursts of the clones whose previous batch came back — no timer
// has to guess when the last clone has submitted.  max_delay_us only bounds
// how long a batch may wait behind a full pipeline before it takes one more
// stream.  Waiters sleep on their batch's generation word (futex: one
// wake-up releases every waiter of the batch together, no mutex to re-take);
// NFFACL_TUNE_BATCH_SPIN lets up to that many spin first (experiments).
#include "batcher.hpp"

#include <linux/futex.h>
#include <time.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>

#include "compile.hpp"
#include "devutil.hpp"
#include "rules.hpp"

using namespace nffacl;
using Clock = std::chrono::steady_clock;

namespace {

// This thread's outstanding-ticket counter per batcher id (the counters
// live in the batcher, nffacl_batcher::owners; the back-pressure bound in
// submit_impl).  A ticket's burst remembers its counter, so a ticket
// collected on another thread still decrements its submitter's count.
thread_local std::unordered_map<uint64_t, std::atomic<int64_t> *> t_own_tickets;
std::atomic<uint64_t> g_batcher_ids{1};

// This thread's counter in `b` (under b->mu).
std::atomic<int64_t> *own_counter(nffacl_batcher *b) {
    auto it = t_own_tickets.find(b->id);
    if (it != t_own_tickets.end()) return it->second;
    b->owners.emplace_back(new std::atomic<int64_t>(0));
    std::atomic<int64_t> *c = b->owners.back().get();
    t_own_tickets.emplace(b->id, c);
    return c;
}


// Mapped (device-addressable) and coherent (fine-grained): the GPU reads the
// slots the CPU just wrote and the CPU reads the verdicts, with no cache
// maintenance between batches.
constexpr unsigned kHostFlags = hipHostMallocMapped | hipHostMallocCoherent;

// Batches on the GPU before an open batch waits for one to complete.
constexpr uint32_t kEagerInflight = 2;

// Futex on a batch's generation word (process-private); `rel` bounds the
// sleep (nullptr: none).
void gen_wait(std::atomic<uint32_t> &g, uint32_t seen, const struct timespec *rel = nullptr) {
    static_assert(sizeof(std::atomic<uint32_t>) == sizeof(uint32_t), "futex word");
    (void)syscall(SYS_futex, reinterpret_cast<uint32_t *>(&g), FUTEX_WAIT_PRIVATE, seen, rel, nullptr, 0);
}

// The batch's verdicts are in (or it failed with `status`): release its
// waiters.
void publish_done(BatchBuf &x, int status) {
    x.status.store(status, std::memory_order_relaxed);
    x.done_seq.store(x.seq.load(std::memory_order_relaxed), std::memory_order_release);
    x.gen.fetch_add(1, std::memory_order_release);
    (void)syscall(SYS_futex, reinterpret_cast<uint32_t *>(&x.gen), FUTEX_WAKE_PRIVATE, INT32_MAX, nullptr, nullptr, 0);
}

void release_buffers(nffacl_batcher *b) {
    if (!b->bufs) return;
    for (uint32_t i = 0; i < b->nbuf; ++i) {
        BatchBuf &x = b->bufs[i];
        if (x.h_slots) (void)hipHostFree(x.h_slots);
        if (x.h_port) (void)hipHostFree(x.h_port);
        if (x.stream) (void)hipStreamDestroy(x.stream);
        if (x.done) (void)hipEventDestroy(x.done);
    }
}

// Under b->mu.  Seal the open buffer and move producers to the next one.
void seal_open(nffacl_batcher *b) {
    BatchBuf &x = b->bufs[b->open_idx];
    x.state = BatchBuf::SEALED;
    if (x.count < b->max_batch) ++b->timeouts;  // shipped before it filled
    b->open_idx = (b->open_idx + 1) % b->nbuf;
    b->cv_work.notify_one();
    b->cv_free.notify_all();  // producers parked on the old open_idx re-check
}

// Under b->mu: a buffer left the busy set.
void free_buffer(nffacl_batcher *b, BatchBuf &x) {
    x.state = BatchBuf::FREE;
    --b->busy;
    b->cv_free.notify_all();
    b->cv_work.notify_one();  // the launcher's eager rule counts busy buffers
}

// Under b->mu: ship bufs[launch_idx] (SEALED).  Drops the lock while launching.
void launch_one(nffacl_batcher *b, std::unique_lock<std::mutex> &lk) {
    const uint32_t i = b->launch_idx;
    BatchBuf &x = b->bufs[i];
    const uint32_t n = x.count;
    b->launch_idx = (i + 1) % b->nbuf;
    ++b->inflight_n;
    const bool inject = b->fail_at != 0 && ++b->launch_no == b->fail_at;
    lk.unlock();
    while (x.written.load(std::memory_order_acquire) < n) std::this_thread::yield();  // copies in progress
    // zero-copy: the kernel reads the mapped slots and writes the mapped ports
    hipError_t e = hipSuccess;
    int st = NFFACL_OK;
    if (inject) {
        set_last_error("batcher launch: injected failure (NFFACL_TUNE_BATCH_FAIL_AT)");
        st = NFFACL_ERR_HIP;
    } else if (x.table) {  // the submitters' rule set (alive until they have waited)
        st = launch_slots(b->eng, x.table, x.d_slots, b->stride, n, x.d_port, nullptr, x.stream);
    } else {
        const TablePtr t = acquire_table(b->eng);  // held while enqueued; the launch records its use
        st = t ? launch_slots(b->eng, t.get(), x.d_slots, b->stride, n, x.d_port, nullptr, x.stream)
               : NFFACL_ERR_INVALID_ARG;
    }
    if (st == NFFACL_OK) e = hipEventRecord(x.done, x.stream);
    lk.lock();
    if (e != hipSuccess || st != NFFACL_OK) {
        if (e != hipSuccess) set_last_error(std::string("batcher launch: ") + hipGetErrorString(e));
        --b->inflight_n;
        ++b->failed;
        x.state = BatchBuf::DONE;  // wake this batch's waiters with the error; later batches are unaffected
        publish_done(x, st != NFFACL_OK ? st : NFFACL_ERR_HIP);
        if (x.readers.load(std::memory_order_acquire) == 0) free_buffer(b, x);
        return;
    }
    x.state = BatchBuf::LAUNCHED;
    ++b->batches;
    b->packets += n;
    b->inflight.push_back(i);
    b->cv_inflight.notify_one();
}

void launcher_main(nffacl_batcher *b) {
    (void)hipSetDevice(b->eng->device);
    (void)prctl(PR_SET_TIMERSLACK, 1000UL);  // µs-scale deadlines, not the default 50 µs slack
    std::unique_lock<std::mutex> lk(b->mu);
    while (true) {
        BatchBuf &x = b->bufs[b->launch_idx];
        if (x.state == BatchBuf::SEALED) {
            launch_one(b, lk);
            continue;
        }
        if (x.state == BatchBuf::OPEN && x.count > 0 && !b->hold) {
            // open_idx == launch_idx here.  Eager: fewer than kEagerInflight
            // batches on the GPU and a free buffer behind this one (so a
            // thread's unwaited tickets fill whole batches: they may hold
            // nbuf - 1 of them).  Late: its first burst has waited max_delay
            // — it ships however busy the other buffers are (held by tickets
            // nobody has collected yet, in any wait order); producers then
            // wait for a buffer (back-pressure).
            const bool room = b->inflight_n < kEagerInflight && b->busy + 2 <= b->nbuf;
            const auto deadline = x.opened + b->max_delay;
            if (b->stop || room || Clock::now() >= deadline) {
                seal_open(b);
                continue;
            }
            b->cv_work.wait_until(lk, deadline);  // a completion, a freed buffer, or the deadline
            continue;
        }
        if (b->stop) {
            if (x.state == BatchBuf::OPEN && x.count > 0) {  // held batch at shutdown: ship it
                seal_open(b);
                continue;
            }
            break;
        }
        b->cv_work.wait(lk);
    }
    b->launcher_done = true;
    b->cv_inflight.notify_all();
}

void completer_main(nffacl_batcher *b) {
    (void)hipSetDevice(b->eng->device);
    (void)prctl(PR_SET_TIMERSLACK, 1000UL);
    std::unique_lock<std::mutex> lk(b->mu);
    while (true) {
        b->cv_inflight.wait(lk, [&] { return !b->inflight.empty() || b->launcher_done; });
        if (b->inflight.empty()) break;
        const uint32_t i = b->inflight.front();
        lk.unlock();
        hipError_t e;
        while ((e = hipEventQuery(b->bufs[i].done)) == hipErrorNotReady) std::this_thread::yield();  // poll: no interrupt wake-up latency
        BatchBuf &x = b->bufs[i];
        if (e != hipSuccess) set_last_error(std::string("batcher completion: ") + hipGetErrorString(e));
        publish_done(x, e == hipSuccess ? NFFACL_OK : NFFACL_ERR_HIP);
        lk.lock();
        b->inflight.pop_front();
        --b->inflight_n;
        x.state = BatchBuf::DONE;
        if (x.readers.load(std::memory_order_acquire) == 0) free_buffer(b, x);
        b->cv_work.notify_one();  // the pipeline has room: the open batch may ship
    }
}

int create_impl(nffacl_engine *eng, bool own, uint32_t stride, uint32_t max_batch, uint32_t max_delay_us,
                uint32_t nbuf, nffacl_batcher **out) {
    nffacl_batcher *b = new (std::nothrow) nffacl_batcher();
    if (!b) return NFFACL_ERR_NOMEM;
    b->id = g_batcher_ids.fetch_add(1, std::memory_order_relaxed);
    b->eng = eng;
    b->own_eng = own;
    b->stride = stride;
    b->max_batch = max_batch;
    b->max_delay = std::chrono::microseconds(max_delay_us);
    b->nbuf = nbuf;
    auto fail = [&](int st) {
        release_buffers(b);
        if (b->own_eng) nffacl_engine_destroy(b->eng);
        delete b;
        return st;
    };
    // Waiters sleep on the batch's futex word at once by default: spinning
    // (sched_yield loops) was slower at every fan-in measured on a 16-CPU
    // share — one thread × 32: 0.98-1.09 Mpps spinning (up to share − 3
    // spinners) vs 1.25-1.35 sleeping (p50 22-24 µs); 32 × 32: 6.9-7.0 vs
    // 8.7-9.1; 64 × 32: 3.9-5.0 vs 5.6-5.8 (profiles/r2_batcher/spin*.jsonl).
    b->spin_limit = 0;
    {  // experiment / test knobs, read once, here
        long v = 0;
        bool set = false;
        std::string err;
        if (!env_knob("NFFACL_TUNE_BATCH_SPIN", 0, 1024, v, set, err)) {
            set_last_error(err);
            return fail(NFFACL_ERR_INVALID_ARG);
        }
        if (set) b->spin_limit = static_cast<uint32_t>(v);
        if (!env_knob("NFFACL_TUNE_BATCH_FAIL_AT", 1, 1L << 40, v, set, err)) {
            set_last_error(err);
            return fail(NFFACL_ERR_INVALID_ARG);
        }
        if (set) b->fail_at = static_cast<uint64_t>(v);
        if (!env_knob("NFFACL_TUNE_BATCH_HOLD", 0, 1, v, set, err)) {
            set_last_error(err);
            return fail(NFFACL_ERR_INVALID_ARG);
        }
        if (set) b->hold = v != 0;
        if (!env_knob("NFFACL_TUNE_BATCH_SUBMIT_MS", 1, 60000, v, set, err)) {
            set_last_error(err);
            return fail(NFFACL_ERR_INVALID_ARG);
        }
        if (set) b->submit_bound = std::chrono::milliseconds(v);
        if (!env_knob("NFFACL_TUNE_BATCH_FOREIGN_MS", 1, 600000, v, set, err)) {
            set_last_error(err);
            return fail(NFFACL_ERR_INVALID_ARG);
        }
        if (set) b->foreign_bound = std::chrono::milliseconds(v);
    }
    b->bufs.reset(new (std::nothrow) BatchBuf[nbuf]);
    if (!b->bufs) return fail(NFFACL_ERR_NOMEM);
    for (uint32_t i = 0; i < nbuf; ++i) {
        BatchBuf &x = b->bufs[i];
        x.claimed.reset(new (std::nothrow) std::atomic<uint64_t>[max_batch]);
        x.owner.reset(new (std::nothrow) std::atomic<int64_t> *[max_batch]);
        if (!x.claimed || !x.owner) return fail(NFFACL_ERR_NOMEM);
        for (uint32_t k = 0; k < max_batch; ++k) {
            x.claimed[k].store(0, std::memory_order_relaxed);
            x.owner[k] = nullptr;
        }
        hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&x.h_slots), size_t(max_batch) * stride, kHostFlags);
        if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&x.h_port), size_t(max_batch) * 4, kHostFlags);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&x.d_slots), x.h_slots, 0);
        if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&x.d_port), x.h_port, 0);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&x.stream, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&x.done, hipEventDisableTiming);
        if (e != hipSuccess) {
            set_last_error(std::string("batcher buffers: ") + hipGetErrorString(e));
            return fail(NFFACL_ERR_HIP);
        }
    }
    b->launcher = std::thread(launcher_main, b);
    b->completer = std::thread(completer_main, b);
    *out = b;
    return NFFACL_OK;
}

// `table`: the rule set's table for every burst (nullptr: the engine's active
// table at launch).
int submit_impl(nffacl_batcher *b, DevTable *table, const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                nffacl_ticket *ticket) {
    if (!b || !ticket || (n && !frames) || n > b->max_batch) return NFFACL_ERR_INVALID_ARG;
    *ticket = nffacl_ticket{0, 0, 0, 0, 0};
    if (n == 0) return NFFACL_OK;
    if (!table && b->own_eng) return NFFACL_ERR_INVALID_ARG;  // a device batcher has no table of its own
    std::unique_lock<std::mutex> lk(b->mu);
    BatchBuf *x = nullptr;
    uint32_t off = 0, burst = 0;
    Clock::time_point first_wait{};  // set at the first back-pressure wait
    while (true) {
        if (b->stop) return NFFACL_ERR_INVALID_ARG;
        BatchBuf &cur = b->bufs[b->open_idx];
        if (cur.state == BatchBuf::FREE) {
            cur.state = BatchBuf::OPEN;
            ++b->busy;
            cur.seq.store(b->next_seq++, std::memory_order_relaxed);
            cur.count = 0;
            cur.bursts = 0;
            cur.table = table;
            cur.status.store(NFFACL_OK, std::memory_order_relaxed);
            cur.readers.store(0, std::memory_order_relaxed);
            cur.written.store(0, std::memory_order_relaxed);
        } else if (cur.state != BatchBuf::OPEN) {
            // every buffer busy: back-pressure.  Buffers whose batches are
            // done stay busy until their tickets are collected; when some of
            // those tickets are this caller's own (submitted, not yet waited
            // for) no amount of waiting may free one, so that wait is bounded
            // by submit_bound.  A caller holding no ticket waits for the
            // other threads' batches (a GPU shared with resident consumers,
            // a first launch) up to foreign_bound.
            const auto now = Clock::now();
            if (first_wait == Clock::time_point{}) first_wait = now;
            const bool self = own_counter(b)->load(std::memory_order_acquire) > 0;
            const auto give_up = first_wait + (self ? b->submit_bound : b->foreign_bound);
            if (now >= give_up) {
                set_last_error(self ? "batcher submit: every buffer holds bursts not yet waited for (this thread's own)"
                                    : "batcher submit: no buffer freed within the bound");
                return NFFACL_ERR_TIMEOUT;
            }
            b->cv_free.wait_until(lk, std::min(give_up, now + std::chrono::milliseconds(50)));
            continue;
        }
        if (cur.count > 0 && cur.table != table) {  // another rule set: the next batch
            seal_open(b);
            continue;
        }
        cur.table = table;
        if (cur.count + n > b->max_batch) {
            seal_open(b);
            continue;
        }
        x = &cur;
        off = cur.count;
        burst = cur.bursts++;
        cur.owner[burst] = own_counter(b);
        cur.owner[burst]->fetch_add(1, std::memory_order_acq_rel);
        if (off == 0) cur.opened = Clock::now();
        cur.count += n;
        cur.readers.fetch_add(1, std::memory_order_relaxed);
        ++b->bursts;
        *ticket = nffacl_ticket{cur.seq.load(std::memory_order_relaxed), b->open_idx, off, n, burst};
        if (cur.count == b->max_batch) seal_open(b);
        else if (off == 0) b->cv_work.notify_one();  // a batch to ship
        break;
    }
    lk.unlock();
    uint8_t *dst = x->h_slots + size_t(off) * b->stride;
    for (uint32_t i = 0; i < n; ++i, dst += b->stride) {
        const uint32_t len = lens ? std::min(lens[i], b->stride) : b->stride;
        if (len) std::memcpy(dst, frames[i], len);
        if (len < b->stride) std::memset(dst + len, 0, b->stride - len);
    }
    x->written.fetch_add(n, std::memory_order_release);
    return NFFACL_OK;
}

// timeout_us == 0: no bound.
int wait_impl(nffacl_batcher *b, const nffacl_ticket *t, uint32_t *ports, uint64_t timeout_us) {
    if (!b || !t) return NFFACL_ERR_INVALID_ARG;
    if (t->n == 0) return NFFACL_OK;
    if (t->buf >= b->nbuf || t->reserved >= b->max_batch) return NFFACL_ERR_INVALID_ARG;
    BatchBuf &x = b->bufs[t->buf];
    auto done = [&] { return x.done_seq.load(std::memory_order_acquire) == t->seq; };
    // optionally spin first, without locks (NFFACL_TUNE_BATCH_SPIN); then sleep
    if (!done()) {
        if (b->spinners.fetch_add(1, std::memory_order_acq_rel) < b->spin_limit) {
            const auto spin_until = Clock::now() + std::chrono::microseconds(200);
            while (!done() && Clock::now() < spin_until) std::this_thread::yield();
        }
        b->spinners.fetch_sub(1, std::memory_order_acq_rel);
    }
    if (!done()) {
        // stale ticket (its buffer was recycled): no mutex on this path — at
        // 64 waiters per batch the lock convoy cost more than the wait; a
        // buffer cannot be recycled while one of its bursts still waits
        if (x.seq.load(std::memory_order_acquire) != t->seq) return NFFACL_ERR_INVALID_ARG;
        const auto deadline = Clock::now() + std::chrono::microseconds(timeout_us);
        while (true) {
            const uint32_t g = x.gen.load(std::memory_order_acquire);
            if (done()) break;
            if (timeout_us == 0) {
                gen_wait(x.gen, g);  // returns at once if the generation moved on
                continue;
            }
            const auto now = Clock::now();
            if (now >= deadline) return NFFACL_ERR_TIMEOUT;  // ticket still valid: wait again later
            const auto left = std::chrono::duration_cast<std::chrono::nanoseconds>(deadline - now).count();
            struct timespec rel;
            rel.tv_sec = static_cast<time_t>(left / 1000000000);
            rel.tv_nsec = static_cast<long>(left % 1000000000);
            gen_wait(x.gen, g, &rel);
        }
    }
    // collect this burst exactly once (a second wait on the ticket would
    // free the buffer under other bursts)
    if (x.claimed[t->reserved].exchange(t->seq, std::memory_order_acq_rel) == t->seq) return NFFACL_ERR_INVALID_ARG;
    if (x.seq.load(std::memory_order_acquire) != t->seq) return NFFACL_ERR_INVALID_ARG;
    const int st = x.status.load(std::memory_order_relaxed);
    if (ports && st == NFFACL_OK) std::memcpy(ports, x.h_port + t->off, size_t(t->n) * 4);
    if (std::atomic<int64_t> *own = x.owner[t->reserved]) own->fetch_sub(1, std::memory_order_acq_rel);  // its submitter's
    if (x.readers.fetch_sub(1, std::memory_order_acq_rel) == 1) {  // the batch's last burst
        std::lock_guard<std::mutex> g(b->mu);
        if (x.state == BatchBuf::DONE) free_buffer(b, x);  // else the completer frees it once it marks it DONE
    }
    return st;
}

}  // namespace

extern "C" {

int nffacl_batcher_create(nffacl_engine *eng, uint32_t stride, uint32_t max_batch, uint32_t max_delay_us,
                          uint32_t nbuf, nffacl_batcher **out) {
    if (!out) return NFFACL_ERR_INVALID_ARG;
    *out = nullptr;
    if (!eng || stride < 64 || stride % 16 != 0 || max_batch < 64 || nbuf < 2) return NFFACL_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(eng->device));
    return create_impl(eng, false, stride, max_batch, max_delay_us, nbuf, out);
}

int nffacl_batcher_create_device(int hip_device, uint32_t stride, uint32_t max_batch, uint32_t max_delay_us,
                                 uint32_t nbuf, nffacl_batcher **out) {
    if (!out) return NFFACL_ERR_INVALID_ARG;
    *out = nullptr;
    if (stride < 64 || stride % 16 != 0 || max_batch < 64 || nbuf < 2) return NFFACL_ERR_INVALID_ARG;
    nffacl_engine *shell = nullptr;
    const int st = engine_shell(hip_device, &shell);
    if (st != NFFACL_OK) return st;
    return create_impl(shell, true, stride, max_batch, max_delay_us, nbuf, out);
}

int nffacl_batcher_submit(nffacl_batcher *b, const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                          nffacl_ticket *ticket) {
    return submit_impl(b, nullptr, frames, lens, n, ticket);
}

int nffacl_batcher_submit_rules(nffacl_batcher *b, const nffacl_rules *rules, const uint8_t *const *frames,
                                const uint32_t *lens, uint32_t n, nffacl_ticket *ticket) {
    if (!b || !rules || !ticket) return NFFACL_ERR_INVALID_ARG;
    int st = NFFACL_OK;
    DevTable *t = rules_table(rules, b->eng->device, st);
    if (!t) return st;
    return submit_impl(b, t, frames, lens, n, ticket);
}

int nffacl_batcher_wait(nffacl_batcher *b, const nffacl_ticket *t, uint32_t *ports) {
    return wait_impl(b, t, ports, 0);
}

int nffacl_batcher_wait_timeout(nffacl_batcher *b, const nffacl_ticket *t, uint32_t *ports, uint64_t timeout_us) {
    return wait_impl(b, t, ports, timeout_us ? timeout_us : 1);
}

int nffacl_batcher_classify(nffacl_batcher *b, const uint8_t *const *frames, const uint32_t *lens, uint32_t n,
                            uint32_t *ports) {
    nffacl_ticket t;
    const int st = nffacl_batcher_submit(b, frames, lens, n, &t);
    if (st != NFFACL_OK) return st;
    return nffacl_batcher_wait(b, &t, ports);
}

int nffacl_batcher_classify_rules(nffacl_batcher *b, const nffacl_rules *rules, const uint8_t *const *frames,
                                  const uint32_t *lens, uint32_t n, uint32_t *ports) {
    nffacl_ticket t;
    const int st = nffacl_batcher_submit_rules(b, rules, frames, lens, n, &t);
    if (st != NFFACL_OK) return st;
    return nffacl_batcher_wait(b, &t, ports);
}

int nffacl_batcher_flush(nffacl_batcher *b) {
    if (!b) return NFFACL_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(b->mu);
    BatchBuf &cur = b->bufs[b->open_idx];
    if (cur.state == BatchBuf::OPEN && cur.count > 0) seal_open(b);
    return NFFACL_OK;
}

int nffacl_batcher_get_stats(nffacl_batcher *b, nffacl_batcher_stats *out) {
    if (!b || !out) return NFFACL_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(b->mu);
    *out = nffacl_batcher_stats{b->batches, b->packets, b->bursts, b->timeouts};
    return NFFACL_OK;
}

void nffacl_batcher_destroy(nffacl_batcher *b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> g(b->mu);
        b->stop = true;
        b->cv_work.notify_all();
        b->cv_free.notify_all();
    }
    if (b->launcher.joinable()) b->launcher.join();
    if (b->completer.joinable()) b->completer.join();
    (void)hipSetDevice(b->eng->device);
    release_buffers(b);
    if (b->own_eng) nffacl_engine_destroy(b->eng);
    delete b;
}

}  // extern "C"
