// tables.cpp — see tables.hpp.
#include "tables.hpp"

namespace nffacl {

namespace {

// Run on `dev` and restore the caller's current device afterwards (a table
// can be retired from any thread, e.g. the last classify_host caller).
struct DeviceScope {
    int old = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&old) != hipSuccess) old = -1;
        if (old != dev) (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        if (old >= 0) (void)hipSetDevice(old);
    }
};

}  // namespace

hipError_t TableHome::init(int dev) {
    device = dev;
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMemoryPoolsSupported, dev) == hipSuccess)
        pools = v != 0;
    else
        (void)hipGetLastError();
    return hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
}

void TableHome::reap(bool all) {
    std::lock_guard<std::mutex> g(mu);
    if (graves.empty()) return;
    DeviceScope ds(device);
    size_t keep = 0;
    for (size_t i = 0; i < graves.size(); ++i) {
        Grave &gr = graves[i];
        hipError_t e = hipSuccess;
        if (gr.fence) e = all ? hipEventSynchronize(gr.fence) : hipEventQuery(gr.fence);
        else if (stream) e = hipStreamSynchronize(stream);
        if (e == hipErrorNotReady) {
            graves[keep++] = std::move(gr);
            continue;
        }
        // fired (or failed, in which case nothing is left to wait for)
        if (gr.blob) (void)hipFree(gr.blob);
        for (hipEvent_t ev : gr.evs) (void)hipEventDestroy(ev);
        if (gr.fence) (void)hipEventDestroy(gr.fence);
    }
    graves.resize(keep);
}

void TableHome::shutdown() {
    if (!stream) return;
    {
        DeviceScope ds(device);
        (void)hipStreamSynchronize(stream);
    }
    reap(true);
    DeviceScope ds(device);
    (void)hipStreamDestroy(stream);
    stream = nullptr;
}

hipError_t DeviceBlob::note_use(hipStream_t s) {
    std::lock_guard<std::mutex> g(use_mu_);
    for (auto &u : uses_)
        if (u.first == s) return hipEventRecord(u.second, s);
    if (uses_.size() >= 16) {  // streams come and go: drop entries whose work has completed
        size_t keep = 0;
        for (size_t i = 0; i < uses_.size(); ++i) {
            if (hipEventQuery(uses_[i].second) == hipErrorNotReady) {
                uses_[keep++] = uses_[i];
            } else {
                (void)hipEventDestroy(uses_[i].second);
            }
        }
        uses_.resize(keep);
    }
    hipEvent_t ev = nullptr;
    hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) return e;
    e = hipEventRecord(ev, s);
    if (e != hipSuccess) {
        (void)hipEventDestroy(ev);
        return e;
    }
    uses_.emplace_back(s, ev);
    return hipSuccess;
}

hipError_t DeviceBlob::upload(TableHome *h, const uint32_t *words, size_t n_words) {
    hipError_t e = alloc(h, n_words);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(d_blob, words, bytes, hipMemcpyHostToDevice, h->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    return e;
}

hipError_t DeviceBlob::alloc(TableHome *h, size_t n_words) {
    home = h;
    bytes = n_words * sizeof(uint32_t);
    void *p = nullptr;
    const bool pools = h->pools.load(std::memory_order_acquire);
    hipError_t e = pools ? hipMallocAsync(&p, bytes, h->stream) : hipMalloc(&p, bytes);
    if (e != hipSuccess && pools) {  // pool refused: plain allocation, freed after its fence
        (void)hipGetLastError();
        h->pools.store(false, std::memory_order_release);
        e = hipMalloc(&p, bytes);
    }
    if (e != hipSuccess) return e;
    d_blob = static_cast<uint32_t *>(p);
    return hipSuccess;
}

DeviceBlob::~DeviceBlob() {
    if (!home) {  // never uploaded through a home (nothing can be in flight)
        if (d_blob) (void)hipFree(d_blob);
        for (auto &u : uses_) (void)hipEventDestroy(u.second);
        return;
    }
    DeviceScope ds(home->device);
    TableHome::Grave gr;
    for (auto &u : uses_) {
        (void)hipStreamWaitEvent(home->stream, u.second, 0);
        gr.evs.push_back(u.second);
    }
    if (d_blob) {
        if (!home->pools.load(std::memory_order_acquire) || hipFreeAsync(d_blob, home->stream) != hipSuccess) {
            (void)hipGetLastError();
            gr.blob = d_blob;  // hipFree once the fence has fired
        }
    }
    if (hipEventCreateWithFlags(&gr.fence, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(gr.fence, home->stream) != hipSuccess) {
        (void)hipGetLastError();
        if (gr.fence) (void)hipEventDestroy(gr.fence);
        gr.fence = nullptr;  // reap() then synchronises the home stream instead
    }
    std::lock_guard<std::mutex> g(home->mu);
    home->graves.push_back(std::move(gr));
}

}  // namespace nffacl
