// capi.cpp — the extern "C" boundary of libnffacl (declared in include/nffacl.h).
//
// No exception crosses this boundary; every entry point returns an nffacl
// status and records details retrievable with nffacl_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "devutil.hpp"
#include "engine.hpp"
#include "l2.hpp"
#include "nffacl.h"
#include "compile.hpp"
#include "rules.hpp"

using namespace nffacl;

namespace {

void copy_err(char *dst, size_t len, const std::string &msg) {
    if (!dst || len == 0) return;
    size_t n = std::min(len - 1, msg.size());
    std::memcpy(dst, msg.data(), n);
    dst[n] = '\0';
}

template <class R>
int finish_parse(bool ok, R *r, const ParseError &pe, R **out, char *err, size_t errlen) {
    if (!ok) {
        delete r;
        *out = nullptr;
        std::string msg = pe.message + " (" + std::to_string(-pe.code) + ")";  // NFError.Error()
        copy_err(err, errlen, msg);
        set_last_error(msg);
        return pe.code;
    }
    copy_err(err, errlen, "");
    *out = r;
    return NFFACL_OK;
}

bool read_file(const char *path, std::vector<char> &buf, std::string &msg) {
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        msg = std::string("file error during rules parsing: open ") + path + ": " + std::strerror(errno);
        return false;
    }
    char tmp[1 << 16];
    size_t got;
    while ((got = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
    const bool bad = std::ferror(f) != 0;
    std::fclose(f);
    if (bad) {
        msg = std::string("file error during rules parsing: read ") + path;
        return false;
    }
    return true;
}

template <class R, class Parser>
int load_with(const char *path, R **out, char *err, size_t errlen, Parser parser) {
    if (!path || !out) return NFFACL_ERR_INVALID_ARG;
    *out = nullptr;
    std::vector<char> buf;
    std::string msg;
    if (!read_file(path, buf, msg)) {
        msg += " (12)";
        copy_err(err, errlen, msg);
        set_last_error(msg);
        return NFFACL_ERR_FILE;
    }
    R *r = new (std::nothrow) R();
    if (!r) return NFFACL_ERR_NOMEM;
    ParseError pe;
    bool ok = parser(buf.data(), buf.size(), *r, pe);
    return finish_parse(ok, r, pe, out, err, errlen);
}

template <class R, class Parser>
int parse_with(const char *text, size_t len, R **out, char *err, size_t errlen, Parser parser) {
    if (!out || (!text && len)) return NFFACL_ERR_INVALID_ARG;
    R *r = new (std::nothrow) R();
    if (!r) return NFFACL_ERR_NOMEM;
    ParseError pe;
    bool ok = parser(text ? text : "", len, *r, pe);
    return finish_parse(ok, r, pe, out, err, errlen);
}

// True iff all of [p, p + bytes) is page-locked host memory of ONE
// allocation (DMA-able as a single copy); otherwise the caller stages it.
bool range_is_pinned(const void *p, size_t bytes) {
    if (bytes == 0) return false;
    hipPointerAttribute_t a, b;
    const void *last = static_cast<const uint8_t *>(p) + bytes - 1;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || hipPointerGetAttributes(&b, last) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (a.type != hipMemoryTypeHost || b.type != hipMemoryTypeHost || !a.devicePointer || !b.devicePointer)
        return false;
    // one allocation: its device alias is contiguous over the range
    const uintptr_t da = reinterpret_cast<uintptr_t>(a.devicePointer), db = reinterpret_cast<uintptr_t>(b.devicePointer);
    if (db - da != bytes - 1) return false;
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, a.devicePointer) != hipSuccess) {
        (void)hipGetLastError();
        return false;  // the range cannot be confirmed as ONE allocation: stage it
    }
    const uintptr_t lo = reinterpret_cast<uintptr_t>(base);
    return da >= lo && db < lo + size;
}

}  // namespace

#define HIP_CHECK HIP_TRY

extern "C" {

int nffacl_abi_version(void) { return NFFACL_ABI_VERSION; }

const char *nffacl_last_error(void) { return last_error(); }

const char *nffacl_strerror(int s) {
    switch (s) {
    case NFFACL_OK: return "ok";
    case NFFACL_ERR_PARSE_RULE_JSON: return "JSON error during rules parsing (ParseRuleJSONErr)";
    case NFFACL_ERR_FILE: return "file error during rules parsing (FileErr)";
    case NFFACL_ERR_PARSE_RULE: return "Incomplete 5-tuple for rule parsing (ParseRuleErr)";
    case NFFACL_ERR_INCORRECT_ARG_IN_RULES: return "incorrect argument in rules (IncorrectArgInRules)";
    case NFFACL_ERR_INCORRECT_RULE: return "incorrect rule result (IncorrectRule)";
    case NFFACL_ERR_INVALID_ARG: return "invalid argument";
    case NFFACL_ERR_NOMEM: return "out of memory";
    case NFFACL_ERR_HIP: return "HIP runtime error";
    case NFFACL_ERR_NO_DEVICE: return "no HIP device";
    case NFFACL_ERR_UNSUPPORTED: return "unsupported";
    case NFFACL_ERR_TIMEOUT: return "timed out";
    default: return "unknown status";
    }
}

// ---- rules -----------------------------------------------------------------

int nffacl_rules_load_text(const char *path, nffacl_rules **out, char *err, size_t errlen) {
    return load_with(path, out, err, errlen, parse_text_table);
}

int nffacl_rules_parse_text(const char *text, size_t len, nffacl_rules **out, char *err,
                            size_t errlen) {
    return parse_with(text, len, out, err, errlen, parse_text_table);
}

int nffacl_rules_load_json(const char *path, nffacl_rules **out, char *err, size_t errlen) {
    return load_with(path, out, err, errlen, parse_json);
}

int nffacl_rules_parse_json(const char *text, size_t len, nffacl_rules **out, char *err,
                            size_t errlen) {
    return parse_with(text, len, out, err, errlen, parse_json);
}

int nffacl_rules_from_arrays(const nffacl_rule4 *r4, size_t n4, const nffacl_rule6 *r6, size_t n6,
                             nffacl_rules **out) {
    if (!out || (!r4 && n4) || (!r6 && n6)) return NFFACL_ERR_INVALID_ARG;
    nffacl_rules *r = new (std::nothrow) nffacl_rules();
    if (!r) return NFFACL_ERR_NOMEM;
    r->ip4.assign(r4, r4 + n4);
    r->ip6.assign(r6, r6 + n6);
    *out = r;
    return NFFACL_OK;
}

void nffacl_rules_free(nffacl_rules *rules) {
    if (!rules) return;
    release_rules_tables(rules);  // its device tables retire behind the work that used them
    delete rules;
}

int nffacl_rules_counts(const nffacl_rules *rules, size_t *n4, size_t *n6) {
    if (!rules) return NFFACL_ERR_INVALID_ARG;
    if (n4) *n4 = rules->ip4.size();
    if (n6) *n6 = rules->ip6.size();
    return NFFACL_OK;
}

int nffacl_rules_get4(const nffacl_rules *rules, size_t i, nffacl_rule4 *out) {
    if (!rules || !out || i >= rules->ip4.size()) return NFFACL_ERR_INVALID_ARG;
    *out = rules->ip4[i];
    return NFFACL_OK;
}

int nffacl_rules_get6(const nffacl_rules *rules, size_t i, nffacl_rule6 *out) {
    if (!rules || !out || i >= rules->ip6.size()) return NFFACL_ERR_INVALID_ARG;
    *out = rules->ip6[i];
    return NFFACL_OK;
}

// ---- host-side table compilation ------------------------------------------

int nffacl_table_compile(const nffacl_rules *rules, int algo, uint32_t *blob, uint64_t cap_dwords,
                         nffacl_table_info *info) {
    if (!rules || !info) return NFFACL_ERR_INVALID_ARG;
    CompiledTable ct;
    std::string err;
    CompileOptions opt;  // tooling: the layout knobs are read per call
    if (!CompileOptions::from_env(opt, err)) {
        set_last_error("tuning knob: " + err);
        return NFFACL_ERR_INVALID_ARG;
    }
    if (!compile_table(*rules, algo, opt, ct, err)) {
        set_last_error("compile: " + err);
        return NFFACL_ERR_INVALID_ARG;
    }
    std::memset(info, 0, sizeof(*info));
    info->algo = ct.algo;
    info->blob_dwords = ct.blob.size();
    info->lds_dwords = ct.lds_dwords;
    info->off_params = ct.off_params;
    info->reserved = 0;
    const FamilyIndex *fi[2] = {&ct.idx4, &ct.idx6};
    const uint32_t off_rec[2] = {ct.off_rec4, ct.off_rec6}, n_rec[2] = {ct.n4, ct.n6};
    for (int f = 0; f < 2; ++f) {
        nffacl_family_info &o = info->fam[f];
        o.n_rec = n_rec[f];
        o.off_rec = off_rec[f];
        o.entry_dwords = fi[f]->entry_dwords;
        o.off_resid = fi[f]->off_resid;
        o.n_resid = fi[f]->n_resid;
        o.n_slots = ct.slots_g ? fi[f]->used_slots : std::max(4u, fi[f]->used_slots);
        o.off_ent_base = fi[f]->off_ent_base;
        for (uint32_t k = 0; k < kMaxSlots; ++k) {
            const DimInfo &d = fi[f]->dims[k];
            o.dims[k] = nffacl_dim_info{d.kind, d.shift, d.n_buckets, d.off_dir, d.off_ent, d.n_rules,
                                        d.max_list, d.off_dir16, d.n_ent, d.kind2, d.shift2, d.bits2, d.dir8};
        }
    }
    if (blob) {
        if (cap_dwords < ct.blob.size()) return NFFACL_ERR_INVALID_ARG;
        std::memcpy(blob, ct.blob.data(), ct.blob.size() * sizeof(uint32_t));
    }
    return NFFACL_OK;
}

// ---- engine ----------------------------------------------------------------

}  // extern "C"

namespace nffacl {

int engine_shell(int hip_device, nffacl_engine **out) {
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_last_error("no HIP device visible");
        return NFFACL_ERR_NO_DEVICE;
    }
    if (hip_device < 0 || hip_device >= count) return NFFACL_ERR_INVALID_ARG;
    HIP_CHECK(hipSetDevice(hip_device));
    int pst = prepare_kernels();
    if (pst != NFFACL_OK) return pst;
    nffacl_engine *eng = new (std::nothrow) nffacl_engine();
    if (!eng) return NFFACL_ERR_NOMEM;
    eng->device = hip_device;
    std::string terr;
    if (!Tune::from_env(eng->tune, terr)) {  // read once; never on the launch path
        set_last_error("tuning knob: " + terr);
        delete eng;
        return NFFACL_ERR_INVALID_ARG;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, hip_device) == hipSuccess && cus > 0)
        eng->num_cus = cus;
    hipError_t e = eng->home.init(hip_device);
    if (e != hipSuccess) {
        set_last_error(std::string("engine stream: ") + hipGetErrorString(e));
        delete eng;
        return NFFACL_ERR_HIP;
    }
    if (eng->tune.dyn) {  // (allocated here: a launch may be captured into a graph)
        const size_t bytes = size_t(nffacl_engine::kDynStreams) * kDynBlockWords * sizeof(uint32_t);
        e = hipMalloc(reinterpret_cast<void **>(&eng->d_dyn), bytes);
        if (e == hipSuccess) e = hipMemset(eng->d_dyn, 0, bytes);
        // (the null-stream memset is not ordered before launches on
        // non-blocking streams — torch's, the group's: complete it here)
        if (e == hipSuccess) e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            set_last_error(std::string("pull heads: ") + hipGetErrorString(e));
            nffacl_engine_destroy(eng);
            return NFFACL_ERR_HIP;
        }
    }
    *out = eng;
    return NFFACL_OK;
}

}  // namespace nffacl

extern "C" {

int nffacl_engine_create_ex(int hip_device, const nffacl_rules *rules, int algo, nffacl_engine **out) {
    if (!rules || !out) return NFFACL_ERR_INVALID_ARG;
    *out = nullptr;
    nffacl_engine *eng = nullptr;
    int st = engine_shell(hip_device, &eng);
    if (st != NFFACL_OK) return st;
    eng->algo_req = algo;
    st = upload_table(eng, *rules, eng->active);
    if (st != NFFACL_OK) {
        nffacl_engine_destroy(eng);
        return st;
    }
    *out = eng;
    return NFFACL_OK;
}

int nffacl_engine_create(int hip_device, const nffacl_rules *rules, nffacl_engine **out) {
    return nffacl_engine_create_ex(hip_device, rules, NFFACL_ALGO_AUTO, out);
}

int nffacl_engine_swap_rules(nffacl_engine *eng, const nffacl_rules *rules) {
    if (!eng || !rules) return NFFACL_ERR_INVALID_ARG;
    TablePtr t;
    int st = upload_table(eng, *rules, t);
    if (st != NFFACL_OK) return st;
    {
        std::lock_guard<std::mutex> g(eng->table_mu);
        eng->active.swap(t);
    }
    // `t` is now the previous table: dropping this reference retires it once
    // no launch / host pipeline / batcher holds it any more — its blob is
    // freed stream-ordered behind the completion events of the work enqueued
    // with it (tables.hpp), without blocking any stream.
    t.reset();
    eng->home.reap(false);  // release earlier retirees whose work has completed
    return NFFACL_OK;
}

void nffacl_engine_destroy(nffacl_engine *eng) {
    if (!eng) return;
    (void)hipSetDevice(eng->device);
    // no classification may be running (header contract): the engine's own
    // streams are synchronised, the table retires behind the user streams'
    // recorded work, and home.shutdown() waits for exactly that
    for (int b = 0; b < nffacl_engine::kHostBufs; ++b)
        if (eng->streams[b]) (void)hipStreamSynchronize(eng->streams[b]);
    eng->active.reset();
    eng->home.shutdown();
    for (int b = 0; b < nffacl_engine::kHostBufs; ++b) {
        if (eng->h_stage[b]) (void)hipHostFree(eng->h_stage[b]);
        if (eng->h_port[b]) (void)hipHostFree(eng->h_port[b]);
        if (eng->d_slots[b]) (void)hipFree(eng->d_slots[b]);
        if (eng->streams[b]) (void)hipStreamDestroy(eng->streams[b]);
        if (eng->done[b]) (void)hipEventDestroy(eng->done[b]);
    }
    if (eng->d_dyn) (void)hipFree(eng->d_dyn);
    delete eng;
}

int nffacl_engine_algo(const nffacl_engine *eng) {
    if (!eng) return NFFACL_ERR_INVALID_ARG;
    const TablePtr t = acquire_table(const_cast<nffacl_engine *>(eng));
    return t ? t->meta.algo : NFFACL_ERR_INVALID_ARG;
}

int nffacl_engine_kernel_info(nffacl_engine *eng, nffacl_kernel_info *out) {
    if (!eng || !out) return NFFACL_ERR_INVALID_ARG;
    return slots_kernel_info(eng, out);
}

int nffacl_engine_table_bytes(const nffacl_engine *eng, uint64_t *bytes) {
    if (!eng || !bytes) return NFFACL_ERR_INVALID_ARG;
    const TablePtr t = acquire_table(const_cast<nffacl_engine *>(eng));
    if (!t) return NFFACL_ERR_INVALID_ARG;
    *bytes = t->bytes;
    return NFFACL_OK;
}

// ---- classification ---------------------------------------------------------

static bool flags_ok(uint32_t flags) { return (flags & ~uint32_t(NFFACL_PARSE_VLAN)) == 0; }

int nffacl_classify_device(nffacl_engine *eng, const uint8_t *d_slots, uint32_t stride, uint64_t n,
                           uint32_t *d_port, uint64_t *d_permit_bits, void *stream) {
    return nffacl_classify_device_ex(eng, d_slots, stride, n, d_port, d_permit_bits, stream, 0);
}

int nffacl_classify_device_ex(nffacl_engine *eng, const uint8_t *d_slots, uint32_t stride, uint64_t n,
                              uint32_t *d_port, uint64_t *d_permit_bits, void *stream, uint32_t flags) {
    if (!eng || !flags_ok(flags)) return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    if (!d_slots || stride < 64 || (stride % 16) != 0 ||
        (reinterpret_cast<uintptr_t>(d_slots) % 16) != 0)
        return NFFACL_ERR_INVALID_ARG;
    if (!d_port && !d_permit_bits) return NFFACL_OK;
    HIP_CHECK(hipSetDevice(eng->device));
    const TablePtr t = acquire_table(eng);  // held while the launch is enqueued
    return launch_slots(eng, t.get(), d_slots, stride, n, d_port, d_permit_bits,
                        static_cast<hipStream_t>(stream), flags);
}

int nffacl_classify_frames_device(nffacl_engine *eng, const uint8_t *d_frames, const uint64_t *d_desc,
                                  uint64_t n, uint32_t *d_port, uint64_t *d_permit_bits, void *stream) {
    return nffacl_classify_frames_device_ex(eng, d_frames, d_desc, n, d_port, d_permit_bits, stream, 0);
}

int nffacl_classify_frames_device_ex(nffacl_engine *eng, const uint8_t *d_frames, const uint64_t *d_desc,
                                     uint64_t n, uint32_t *d_port, uint64_t *d_permit_bits, void *stream,
                                     uint32_t flags) {
    if (!eng || !flags_ok(flags)) return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    if (!d_frames || !d_desc || (reinterpret_cast<uintptr_t>(d_frames) % 16) != 0)
        return NFFACL_ERR_INVALID_ARG;
    if (!d_port && !d_permit_bits) return NFFACL_OK;
    HIP_CHECK(hipSetDevice(eng->device));
    const TablePtr t = acquire_table(eng);
    return launch_frames(eng, t.get(), d_frames, d_desc, n, d_port, d_permit_bits,
                         static_cast<hipStream_t>(stream), flags);
}

// Host pipeline buffers, sized to the request: small calls get small pinned
// buffers, large ones stream through `host_bufs` chunks of 2^host_chunk
// packets (one stream each).
static int ensure_host_pipeline(nffacl_engine *eng, uint32_t stride, uint64_t n) {
    const int nb = std::max(2, std::min(eng->tune.host_bufs, int(nffacl_engine::kHostBufs)));
    const size_t cap = size_t(1) << std::max(12, std::min(eng->tune.host_chunk, 24));
    size_t chunk = size_t(1) << 12;
    while (chunk < n && chunk < cap) chunk <<= 1;
    if (eng->chunk >= chunk && eng->staged_stride >= stride && eng->nbufs == nb) return NFFACL_OK;
    if (eng->nbufs == nb) chunk = std::max(chunk, eng->chunk);
    stride = std::max(stride, eng->staged_stride);
    for (int b = 0; b < nffacl_engine::kHostBufs; ++b) {
        if (eng->streams[b]) (void)hipStreamSynchronize(eng->streams[b]);
        if (eng->h_stage[b]) { (void)hipHostFree(eng->h_stage[b]); eng->h_stage[b] = nullptr; }
        if (eng->d_slots[b]) { (void)hipFree(eng->d_slots[b]); eng->d_slots[b] = nullptr; }
        if (eng->h_port[b]) { (void)hipHostFree(eng->h_port[b]); eng->h_port[b] = nullptr; eng->d_hport[b] = nullptr; }
    }
    eng->chunk = 0;
    eng->nbufs = 0;
    for (int b = 0; b < nb; ++b) {
        HIP_CHECK(hipHostMalloc(reinterpret_cast<void **>(&eng->h_stage[b]), chunk * stride, hipHostMallocDefault));
        HIP_CHECK(hipMalloc(reinterpret_cast<void **>(&eng->d_slots[b]), chunk * stride));
        HIP_CHECK(hipHostMalloc(reinterpret_cast<void **>(&eng->h_port[b]), chunk * 4, hipHostMallocMapped));
        HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&eng->d_hport[b]), eng->h_port[b], 0));
        if (!eng->streams[b]) HIP_CHECK(hipStreamCreateWithFlags(&eng->streams[b], hipStreamNonBlocking));
        if (!eng->done[b]) HIP_CHECK(hipEventCreateWithFlags(&eng->done[b], hipEventDisableTiming));
    }
    eng->chunk = chunk;
    eng->nbufs = nb;
    eng->staged_stride = stride;
    return NFFACL_OK;
}

int nffacl_classify_host(nffacl_engine *eng, const uint8_t *h_slots, uint32_t stride, uint64_t n,
                         uint32_t *h_port, uint8_t *h_permit) {
    return nffacl_classify_host_ex(eng, h_slots, stride, n, h_port, h_permit, 0);
}

// Device alias of pinned (mapped) host memory, or nullptr.
static void *host_alias(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

int nffacl_classify_host_ex(nffacl_engine *eng, const uint8_t *h_slots, uint32_t stride, uint64_t n,
                            uint32_t *h_port, uint8_t *h_permit, uint32_t flags) {
    if (!eng || !flags_ok(flags)) return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    if (!h_slots || stride < 64 || (stride % 16) != 0) return NFFACL_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(eng->host_mu);
    HIP_CHECK(hipSetDevice(eng->device));
    int st = ensure_host_pipeline(eng, stride, n);
    if (st != NFFACL_OK) return st;
    const TablePtr t = acquire_table(eng);  // one table for every chunk of this call
    // Input: pinned caller memory (one registered allocation) is read where it
    // lies — by the kernel itself over PCIe (zero-copy: its lane-contiguous
    // 1 KiB loads keep the link busy, no copy engine), or DMA'd chunk by chunk
    // into HBM (NFFACL_TUNE_HOST_DMA=1); pageable input is copied into pinned
    // staging, then DMA'd.  Output: every kernel writes its verdicts over PCIe
    // into mapped pinned memory — the caller's when that is pinned, else the
    // chunk's staging, copied out when the chunk completes.
    const bool pinned_in = range_is_pinned(h_slots, n * stride) && reinterpret_cast<uintptr_t>(h_slots) % 16 == 0;
    const uint8_t *d_host_slots = pinned_in ? static_cast<const uint8_t *>(host_alias(h_slots)) : nullptr;
    const bool zero_copy = d_host_slots && eng->tune.host_dma == 0;
    uint32_t *d_host_port = nullptr;
    if (h_port && range_is_pinned(h_port, n * 4) && reinterpret_cast<uintptr_t>(h_port) % 4 == 0)
        d_host_port = static_cast<uint32_t *>(host_alias(h_port));
    const uint64_t chunk = eng->chunk;
    const int nb = eng->nbufs;
    const uint64_t nchunks = (n + chunk - 1) / chunk;
    uint64_t pending_chunk[nffacl_engine::kHostBufs];
    for (int b = 0; b < nffacl_engine::kHostBufs; ++b) pending_chunk[b] = ~0ull;
    auto drain = [&](int b) -> int {
        if (pending_chunk[b] == ~0ull) return NFFACL_OK;
        HIP_CHECK(hipEventSynchronize(eng->done[b]));
        const uint64_t c = pending_chunk[b];
        const uint64_t first = c * chunk;
        const uint64_t cnt = std::min<uint64_t>(chunk, n - first);
        const uint32_t *res = d_host_port ? h_port + first : eng->h_port[b];
        if (h_port && !d_host_port) std::memcpy(h_port + first, res, cnt * 4);
        if (h_permit)
            for (uint64_t i = 0; i < cnt; ++i) h_permit[first + i] = res[i] != 0;
        pending_chunk[b] = ~0ull;
        return NFFACL_OK;
    };
    for (uint64_t c = 0; c < nchunks; ++c) {
        const int b = static_cast<int>(c % uint64_t(nb));
        if ((st = drain(b)) != NFFACL_OK) return st;
        const uint64_t first = c * chunk;
        const uint64_t cnt = std::min<uint64_t>(chunk, n - first);
        uint32_t *out = d_host_port ? d_host_port + first : eng->d_hport[b];
        const uint8_t *in = nullptr;
        if (zero_copy) {
            in = d_host_slots + first * stride;
        } else {
            const uint8_t *src = h_slots + first * stride;
            if (!pinned_in) {
                std::memcpy(eng->h_stage[b], src, cnt * stride);
                src = eng->h_stage[b];
            }
            HIP_CHECK(hipMemcpyAsync(eng->d_slots[b], src, cnt * stride, hipMemcpyHostToDevice, eng->streams[b]));
            in = eng->d_slots[b];
        }
        st = launch_slots(eng, t.get(), in, stride, cnt, out, nullptr, eng->streams[b], flags);
        if (st != NFFACL_OK) return st;
        HIP_CHECK(hipEventRecord(eng->done[b], eng->streams[b]));
        pending_chunk[b] = c;
    }
    for (uint64_t c = nchunks > uint64_t(nb) ? nchunks - nb : 0; c < nchunks; ++c)  // completion order
        if ((st = drain(static_cast<int>(c % uint64_t(nb)))) != NFFACL_OK) return st;
    return NFFACL_OK;
}

// ---- L2 ACL -------------------------------------------------------------------

int nffacl_l2rules_load_text(const char *path, nffacl_l2rules **out, char *err, size_t errlen) {
    return load_with(path, out, err, errlen, parse_l2_text_table);
}

int nffacl_l2rules_parse_text(const char *text, size_t len, nffacl_l2rules **out, char *err, size_t errlen) {
    return parse_with(text, len, out, err, errlen, parse_l2_text_table);
}

int nffacl_l2rules_load_json(const char *path, nffacl_l2rules **out, char *err, size_t errlen) {
    return load_with(path, out, err, errlen, parse_l2_json);
}

int nffacl_l2rules_parse_json(const char *text, size_t len, nffacl_l2rules **out, char *err, size_t errlen) {
    return parse_with(text, len, out, err, errlen, parse_l2_json);
}

int nffacl_l2rules_from_array(const nffacl_l2_rule *r, size_t n, nffacl_l2rules **out) {
    if (!out || (!r && n)) return NFFACL_ERR_INVALID_ARG;
    nffacl_l2rules *x = new (std::nothrow) nffacl_l2rules();
    if (!x) return NFFACL_ERR_NOMEM;
    x->eth.assign(r, r + n);
    *out = x;
    return NFFACL_OK;
}

void nffacl_l2rules_free(nffacl_l2rules *rules) { delete rules; }

int nffacl_l2rules_count(const nffacl_l2rules *rules, size_t *n) {
    if (!rules || !n) return NFFACL_ERR_INVALID_ARG;
    *n = rules->eth.size();
    return NFFACL_OK;
}

int nffacl_l2rules_get(const nffacl_l2rules *rules, size_t i, nffacl_l2_rule *out) {
    if (!rules || !out || i >= rules->eth.size()) return NFFACL_ERR_INVALID_ARG;
    *out = rules->eth[i];
    return NFFACL_OK;
}

int nffacl_l2_engine_create(int hip_device, const nffacl_l2rules *rules, nffacl_l2engine **out) {
    return nffacl_l2_engine_create_ex(hip_device, rules, NFFACL_ALGO_AUTO, out);
}

static L2TablePtr acquire_l2(nffacl_l2engine *eng) {
    std::lock_guard<std::mutex> g(eng->table_mu);
    return eng->active;
}

int nffacl_l2_engine_algo(const nffacl_l2engine *eng) {
    if (!eng) return NFFACL_ERR_INVALID_ARG;
    const L2TablePtr t = acquire_l2(const_cast<nffacl_l2engine *>(eng));
    return t ? t->meta.algo : NFFACL_ERR_INVALID_ARG;
}

int nffacl_l2_engine_create_ex(int hip_device, const nffacl_l2rules *rules, int algo, nffacl_l2engine **out) {
    if (!rules || !out) return NFFACL_ERR_INVALID_ARG;
    if (algo != NFFACL_ALGO_AUTO && algo != NFFACL_ALGO_LINEAR && algo != NFFACL_ALGO_INDEXED)
        return NFFACL_ERR_INVALID_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_last_error("no HIP device visible");
        return NFFACL_ERR_NO_DEVICE;
    }
    if (hip_device < 0 || hip_device >= count) return NFFACL_ERR_INVALID_ARG;
    HIP_CHECK(hipSetDevice(hip_device));
    int pst = l2_prepare_kernels();
    if (pst != NFFACL_OK) return pst;
    nffacl_l2engine *eng = new (std::nothrow) nffacl_l2engine();
    if (!eng) return NFFACL_ERR_NOMEM;
    eng->device = hip_device;
    eng->algo_req = algo;
    long v = 0;
    bool set = false;
    std::string terr;
    if (!env_knob("NFFACL_TUNE_L2_COAL", 0, 1, v, set, terr)) {  // read once; never on the launch path
        set_last_error("tuning knob: " + terr);
        delete eng;
        return NFFACL_ERR_INVALID_ARG;
    }
    if (set) eng->coal = v != 0;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, hip_device) == hipSuccess && cus > 0)
        eng->num_cus = cus;
    hipError_t e = eng->home.init(hip_device);
    if (e != hipSuccess) {
        set_last_error(std::string("engine stream: ") + hipGetErrorString(e));
        delete eng;
        return NFFACL_ERR_HIP;
    }
    int st = upload_l2(eng, *rules, eng->active);
    if (st != NFFACL_OK) {
        delete eng;
        return st;
    }
    *out = eng;
    return NFFACL_OK;
}

int nffacl_l2_engine_swap_rules(nffacl_l2engine *eng, const nffacl_l2rules *rules) {
    if (!eng || !rules) return NFFACL_ERR_INVALID_ARG;
    L2TablePtr t;
    int st = upload_l2(eng, *rules, t);
    if (st != NFFACL_OK) return st;
    {
        std::lock_guard<std::mutex> g(eng->table_mu);
        eng->active.swap(t);
    }
    t.reset();  // retires the previous table behind its recorded work (tables.hpp)
    eng->home.reap(false);
    return NFFACL_OK;
}

void nffacl_l2_engine_destroy(nffacl_l2engine *eng) {
    if (!eng) return;
    (void)hipSetDevice(eng->device);
    if (eng->stream) (void)hipStreamSynchronize(eng->stream);
    eng->active.reset();
    eng->home.shutdown();
    if (eng->d_slots) (void)hipFree(eng->d_slots);
    if (eng->d_port) (void)hipFree(eng->d_port);
    if (eng->stream) (void)hipStreamDestroy(eng->stream);
    delete eng;
}

int nffacl_l2_classify_device(nffacl_l2engine *eng, const uint8_t *d_slots, uint32_t stride, uint64_t n,
                              uint32_t *d_port, uint64_t *d_permit_bits, void *stream) {
    if (!eng) return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    if (!d_slots || stride < 64 || (stride % 16) != 0 || (reinterpret_cast<uintptr_t>(d_slots) % 16) != 0)
        return NFFACL_ERR_INVALID_ARG;
    if (!d_port && !d_permit_bits) return NFFACL_OK;
    HIP_CHECK(hipSetDevice(eng->device));
    const L2TablePtr t = acquire_l2(eng);
    return l2_launch_slots(eng, t.get(), d_slots, stride, n, d_port, d_permit_bits,
                           static_cast<hipStream_t>(stream));
}

int nffacl_l2_classify_frames_device(nffacl_l2engine *eng, const uint8_t *d_frames, const uint64_t *d_desc,
                                     uint64_t n, uint32_t *d_port, uint64_t *d_permit_bits, void *stream) {
    if (!eng) return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    if (!d_frames || !d_desc || (reinterpret_cast<uintptr_t>(d_frames) % 16) != 0) return NFFACL_ERR_INVALID_ARG;
    if (!d_port && !d_permit_bits) return NFFACL_OK;
    HIP_CHECK(hipSetDevice(eng->device));
    const L2TablePtr t = acquire_l2(eng);
    return l2_launch_frames(eng, t.get(), d_frames, d_desc, n, d_port, d_permit_bits,
                            static_cast<hipStream_t>(stream));
}

int nffacl_l2_classify_host(nffacl_l2engine *eng, const uint8_t *h_slots, uint32_t stride, uint64_t n,
                            uint32_t *h_port, uint8_t *h_permit) {
    if (!eng) return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    if (!h_slots || stride < 64 || (stride % 16) != 0) return NFFACL_ERR_INVALID_ARG;
    if (!h_port && !h_permit) return NFFACL_OK;
    std::lock_guard<std::mutex> g(eng->host_mu);
    HIP_CHECK(hipSetDevice(eng->device));
    if (!eng->stream) HIP_CHECK(hipStreamCreateWithFlags(&eng->stream, hipStreamNonBlocking));
    if (eng->cap_bytes < n * stride) {
        if (eng->d_slots) (void)hipFree(eng->d_slots);
        eng->d_slots = nullptr;
        eng->cap_bytes = 0;
        HIP_CHECK(hipMalloc(reinterpret_cast<void **>(&eng->d_slots), n * stride));
        eng->cap_bytes = n * stride;
    }
    if (eng->cap_n < n) {
        if (eng->d_port) (void)hipFree(eng->d_port);
        eng->d_port = nullptr;
        eng->cap_n = 0;
        HIP_CHECK(hipMalloc(reinterpret_cast<void **>(&eng->d_port), n * 4));
        eng->cap_n = n;
    }
    std::vector<uint32_t> tmp;
    uint32_t *port = h_port;
    if (!port) {
        tmp.resize(n);
        port = tmp.data();
    }
    HIP_CHECK(hipMemcpyAsync(eng->d_slots, h_slots, n * stride, hipMemcpyHostToDevice, eng->stream));
    const L2TablePtr t = acquire_l2(eng);
    int st = l2_launch_slots(eng, t.get(), eng->d_slots, stride, n, eng->d_port, nullptr, eng->stream);
    if (st != NFFACL_OK) return st;
    HIP_CHECK(hipMemcpyAsync(port, eng->d_port, n * 4, hipMemcpyDeviceToHost, eng->stream));
    HIP_CHECK(hipStreamSynchronize(eng->stream));
    if (h_permit)
        for (uint64_t i = 0; i < n; ++i) h_permit[i] = port[i] != 0;
    return NFFACL_OK;
}

}  // extern "C"
