// group.cpp — one process driving several GPUs of a node (nffacl_group_*,
// nffacl_pick_device), compiled as HIP and linked against RCCL.
//
// The reference scales a flow function by core-pinned clones inside ONE
// process (flow/scheduler.go:283-289 starts a clone per core,
// internal/low/low.go:654-666 pins it), every clone calling
// (*Packet).L3ACLPermit on the same shared *L3Rules (packet/acl.go:495-506).
// A Go host on an 8-GPU node therefore reaches the GPUs through this one
// library instance, not through one process per GPU:
//  * nffacl_local_device() spreads the clones of a NUMA node over ALL of that
//    node's GPUs (the clone's CPU rank among the node's CPUs, modulo the
//    node's device count; stable per thread) — nffacl_pick_device() is the
//    map itself, testable on any topology;
//  * an nffacl_group holds one RCCL communicator per device
//    (ncclCommInitAll), compiles the rule set once on the host, uploads it to
//    the root device and ncclBroadcasts the table image to the others over
//    xGMI; nffacl_group_classify_device() takes a batch resident on the root
//    device, ncclSend/ncclRecv-scatters 64-aligned shards to the other
//    devices (one group call: the root's sends run concurrently over its
//    links), classifies every shard on its own device, and gathers the
//    verdicts (ports and permit words) back into the root's arrays.  All of
//    it is enqueued on the caller's root stream (and the group's per-device
//    streams): the call returns at once, like nffacl_classify_device.
// RCCL is opened (dlopen) by the first nffacl_group_create only, so the
// library itself does not depend on it: single-GPU users need no RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // (types and prototypes only: the calls go through Rccl below)
#include <sched.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "devutil.hpp"
#include "engine.hpp"
#include "nffacl.h"
#include "rules.hpp"

using namespace nffacl;

namespace {

// Current device restored on scope exit (one thread drives every device);
// `ok` false (and the last error set) when the switch failed.
struct OnDevice {
    int prev = 0;
    bool ok = true;
    explicit OnDevice(int dev) {
        (void)hipGetDevice(&prev);
        const hipError_t e = hipSetDevice(dev);
        ok = e == hipSuccess;
        if (!ok) set_last_error(std::string("hipSetDevice(") + std::to_string(dev) + "): " + hipGetErrorString(e));
    }
    ~OnDevice() { (void)hipSetDevice(prev); }
};

// The RCCL entry points the group uses, resolved from librccl at run time.
struct Rccl {
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string err;  // why loading failed ("" = loaded)
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = nullptr;
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1", "/opt/rocm/lib/librccl.so"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (!h) {
            const char *e = dlerror();
            r.err = std::string("RCCL not available: ") + (e ? e : "librccl.so not found");
            return;
        }
        auto sym = [&](auto &fp, const char *name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            if (!fp && r.err.empty()) r.err = std::string("RCCL symbol missing: ") + name;
        };
        sym(r.comm_init_all, "ncclCommInitAll");
        sym(r.comm_destroy, "ncclCommDestroy");
        sym(r.broadcast, "ncclBroadcast");
        sym(r.send, "ncclSend");
        sym(r.recv, "ncclRecv");
        sym(r.group_start, "ncclGroupStart");
        sym(r.group_end, "ncclGroupEnd");
        sym(r.error_string, "ncclGetErrorString");
    });
    return r;
}

// One RCCL group (ncclGroupStart .. ncclGroupEnd) whose calls are all
// checked: the first failing call or device switch is remembered, the group
// is still closed (RCCL requires it), and end() reports the first failure —
// a call rejected inside the group must not leave a peer waiting on a
// receive that was never posted without the caller hearing of it.
struct CheckedGroup {
    const Rccl &R;
    const char *what;
    std::string err;
    bool open = false;
    CheckedGroup(const Rccl &r, const char *w) : R(r), what(w) {
        const ncclResult_t e = R.group_start();
        if (e != ncclSuccess) err = std::string("ncclGroupStart: ") + R.error_string(e);
        open = e == ncclSuccess;
    }
    bool ok() const { return err.empty(); }
    void nccl(ncclResult_t e, const char *call) {
        if (e != ncclSuccess && err.empty()) err = std::string(call) + ": " + R.error_string(e);
    }
    void device(int dev) {
        const hipError_t e = hipSetDevice(dev);
        if (e != hipSuccess && err.empty()) err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    }
    int end() {
        if (open) {
            const ncclResult_t e = R.group_end();
            open = false;
            if (e != ncclSuccess && err.empty()) err = std::string("ncclGroupEnd: ") + R.error_string(e);
        }
        if (err.empty()) return NFFACL_OK;
        set_last_error(std::string(what) + ": " + err);
        return NFFACL_ERR_HIP;
    }
    ~CheckedGroup() {
        if (open) (void)R.group_end();
    }
};

// CPU -> NUMA node map of this host (sysfs), built once.
const std::vector<int> &cpu_nodes() {
    static std::vector<int> map;
    static std::once_flag once;
    std::call_once(once, [] {
        for (int node = 0; node < 1024; ++node) {
            const std::string path = "/sys/devices/system/node/node" + std::to_string(node) + "/cpulist";
            FILE *f = std::fopen(path.c_str(), "r");
            if (!f) {
                if (node > 64) break;  // (node numbers may have gaps; stop well past the last)
                continue;
            }
            char buf[8192] = {0};
            const size_t got = std::fread(buf, 1, sizeof buf - 1, f);
            std::fclose(f);
            buf[got] = 0;
            // "0-63,128-191"
            for (char *p = buf; *p;) {
                char *end = nullptr;
                const long a = std::strtol(p, &end, 10);
                if (end == p) break;
                long b = a;
                p = end;
                if (*p == '-') b = std::strtol(p + 1, &p, 10);
                for (long c = a; c <= b && c < (1 << 16); ++c) {
                    if (static_cast<size_t>(c) >= map.size()) map.resize(c + 1, -1);
                    map[c] = node;
                }
                while (*p == ',' || *p == '\n' || *p == ' ') ++p;
            }
        }
    });
    return map;
}

}  // namespace

struct nffacl_group {
    int n = 0;
    std::vector<int> devs;
    std::vector<ncclComm_t> comms;
    std::vector<nffacl_engine *> engs;   // launch shape + table home per device (engine shells)
    std::vector<TablePtr> tabs;          // the rule set's table on every device
    std::vector<hipStream_t> streams;    // devices 1..n-1 (device 0: the caller's stream)
    std::vector<uint8_t *> d_in;         // shard staging per device (1..n-1)
    std::vector<uint32_t *> d_out;
    std::vector<uint64_t *> d_perm;
    std::vector<size_t> cap;             // packets the staging holds
    uint32_t cap_stride = 0;
    std::mutex mu;                       // collectives on shared communicators: one call at a time
};

namespace {

void group_release(nffacl_group *g) {
    for (int i = 0; i < g->n; ++i) {
        OnDevice od(g->devs[i]);
        if (i > 0 && i < static_cast<int>(g->streams.size()) && g->streams[i]) {
            (void)hipStreamSynchronize(g->streams[i]);
            (void)hipStreamDestroy(g->streams[i]);
        }
        if (i < static_cast<int>(g->d_in.size())) {
            if (g->d_in[i]) (void)hipFree(g->d_in[i]);
            if (g->d_out[i]) (void)hipFree(g->d_out[i]);
            if (g->d_perm[i]) (void)hipFree(g->d_perm[i]);
        }
    }
    for (ncclComm_t c : g->comms)
        if (c) (void)rccl().comm_destroy(c);
    g->tabs.clear();  // retired stream-ordered through each device's table home
    for (nffacl_engine *e : g->engs)
        if (e) nffacl_engine_destroy(e);
    delete g;
}

// Staging for shards of `per` packets of `stride` bytes on devices 1..n-1.
int ensure_staging(nffacl_group *g, size_t per, uint32_t stride) {
    for (int i = 1; i < g->n; ++i) {
        if (g->cap[i] >= per && g->cap_stride >= stride) continue;
        OnDevice od(g->devs[i]);
        if (!od.ok) return NFFACL_ERR_HIP;
        HIP_TRY(hipStreamSynchronize(g->streams[i]));  // the previous call's use of the old buffers
        if (g->d_in[i]) (void)hipFree(g->d_in[i]);
        if (g->d_out[i]) (void)hipFree(g->d_out[i]);
        if (g->d_perm[i]) (void)hipFree(g->d_perm[i]);
        g->d_in[i] = nullptr;
        g->d_out[i] = nullptr;
        g->d_perm[i] = nullptr;
        g->cap[i] = 0;
        const size_t words = (per + 63) / 64;
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&g->d_in[i]), per * std::max(stride, g->cap_stride)));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&g->d_out[i]), per * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(reinterpret_cast<void **>(&g->d_perm[i]), words * sizeof(uint64_t)));
        g->cap[i] = per;
    }
    g->cap_stride = std::max(g->cap_stride, stride);
    return NFFACL_OK;
}

}  // namespace

extern "C" {

int nffacl_pick_device(int cpu, const int *cpu_node, int n_cpus, const int *dev_node, int n_devs) {
    if (n_devs <= 0 || !dev_node || (n_cpus > 0 && !cpu_node) || n_cpus < 0) return NFFACL_ERR_INVALID_ARG;
    const int node = cpu >= 0 && cpu < n_cpus ? cpu_node[cpu] : -1;
    // the node's devices, in device order (none: every device)
    int local[4096];
    int nl = 0;
    for (int d = 0; d < n_devs && nl < 4096; ++d)
        if (node >= 0 && dev_node[d] == node) local[nl++] = d;
    if (nl == 0)
        for (int d = 0; d < n_devs && nl < 4096; ++d) local[nl++] = d;
    // the CPU's rank among its node's CPUs (unknown node: the CPU number)
    int rank = cpu >= 0 ? cpu : 0;
    if (node >= 0) {
        rank = 0;
        for (int c = 0; c < cpu; ++c) rank += cpu_node[c] == node ? 1 : 0;
    }
    return local[rank % nl];
}

int nffacl_local_device(void) {
    thread_local int cached = -1;  // stable per thread: its first call decides
    if (cached >= 0) return cached;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        return NFFACL_ERR_NO_DEVICE;
    }
    std::vector<int> dn(count, -1);
    for (int d = 0; d < count; ++d) {
        const int node = nffacl_device_numa_node(d);
        dn[d] = node >= 0 ? node : -1;
    }
    const std::vector<int> &cn = cpu_nodes();
    const int cpu = sched_getcpu();
    const int d = nffacl_pick_device(cpu, cn.data(), static_cast<int>(cn.size()), dn.data(), count);
    cached = d >= 0 ? d : 0;
    return cached;
}

int nffacl_group_shard(uint64_t n, int n_devices, int i, uint64_t *off, uint64_t *len) {
    if (!off || !len || n_devices <= 0 || n_devices > 64 || i < 0 || i >= n_devices || n > (uint64_t(1) << 48))
        return NFFACL_ERR_INVALID_ARG;
    // 64-aligned shards (a permit word never straddles two devices); the
    // root keeps the first, trailing devices may get none (n < 64 (N - 1))
    const uint64_t per = ((n + uint64_t(n_devices) - 1) / uint64_t(n_devices) + 63) / 64 * 64;
    *off = std::min<uint64_t>(n, per * uint64_t(i));
    *len = std::min<uint64_t>(n, per * uint64_t(i + 1)) - *off;
    return NFFACL_OK;
}

int nffacl_group_create(const int *hip_devices, int n, const nffacl_rules *rules, nffacl_group **out) {
    if (!out) return NFFACL_ERR_INVALID_ARG;
    *out = nullptr;
    if (!hip_devices || n <= 0 || n > 64 || !rules) return NFFACL_ERR_INVALID_ARG;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_last_error("no HIP device visible");
        return NFFACL_ERR_NO_DEVICE;
    }
    for (int i = 0; i < n; ++i) {
        if (hip_devices[i] < 0 || hip_devices[i] >= count) return NFFACL_ERR_INVALID_ARG;
        for (int j = 0; j < i; ++j)
            if (hip_devices[j] == hip_devices[i]) return NFFACL_ERR_INVALID_ARG;  // one rank per device
    }
    const Rccl &R = rccl();
    if (!R.err.empty()) {
        set_last_error(R.err);
        return NFFACL_ERR_HIP;
    }
    nffacl_group *g = new (std::nothrow) nffacl_group();
    if (!g) return NFFACL_ERR_NOMEM;
    g->n = n;
    g->devs.assign(hip_devices, hip_devices + n);
    g->engs.assign(n, nullptr);
    g->streams.assign(n, nullptr);
    g->d_in.assign(n, nullptr);
    g->d_out.assign(n, nullptr);
    g->d_perm.assign(n, nullptr);
    g->cap.assign(n, 0);
    auto fail = [&](int st) {
        group_release(g);
        return st;
    };
    for (int i = 0; i < n; ++i) {
        const int st = engine_shell(g->devs[i], &g->engs[i]);
        if (st != NFFACL_OK) return fail(st);
        if (i > 0) {
            OnDevice od(g->devs[i]);
            if (!od.ok) return fail(NFFACL_ERR_HIP);
            if (hipStreamCreateWithFlags(&g->streams[i], hipStreamNonBlocking) != hipSuccess) {
                set_last_error("group stream");
                return fail(NFFACL_ERR_HIP);
            }
        }
    }
    g->comms.assign(n, nullptr);
    {
        const ncclResult_t e = R.comm_init_all(g->comms.data(), n, g->devs.data());
        if (e != ncclSuccess) {
            set_last_error(std::string("ncclCommInitAll: ") + R.error_string(e));
            g->comms.clear();
            return fail(NFFACL_ERR_HIP);
        }
    }
    // compile once on the host; upload to the root, broadcast the image
    std::vector<uint32_t> words;
    for (int i = 0; i < n; ++i) g->tabs.push_back(std::make_shared<DevTable>());
    int st = compile_words(*rules, g->engs[0]->algo_req, g->engs[0]->tune.copt, *g->tabs[0], words);
    if (st != NFFACL_OK) return fail(st);
    for (int i = 0; i < n; ++i) {
        OnDevice od(g->devs[i]);
        if (!od.ok) return fail(NFFACL_ERR_HIP);
        DevTable &t = *g->tabs[i];
        if (i > 0) {
            t.meta = g->tabs[0]->meta;
            t.svc_kind = g->tabs[0]->svc_kind;
        }
        const hipError_t e = i == 0 ? t.upload(&g->engs[i]->home, words.data(), words.size())
                                    : t.alloc(&g->engs[i]->home, words.size());
        if (e != hipSuccess) {
            set_last_error(std::string("group table: ") + hipGetErrorString(e));
            return fail(e == hipErrorOutOfMemory ? NFFACL_ERR_NOMEM : NFFACL_ERR_HIP);
        }
    }
    if (n > 1) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        CheckedGroup grp(R, "table broadcast");
        for (int i = 0; i < n && grp.ok(); ++i) {
            grp.device(g->devs[i]);
            if (grp.ok())
                grp.nccl(R.broadcast(g->tabs[0]->d_blob, g->tabs[i]->d_blob, words.size(), ncclUint32, 0, g->comms[i],
                                     g->engs[i]->home.stream),
                         "ncclBroadcast");
        }
        st = grp.end();
        (void)hipSetDevice(prev);
        if (st != NFFACL_OK) return fail(st);
    }
    for (int i = 0; i < n; ++i) {
        OnDevice od(g->devs[i]);
        if (!od.ok) return fail(NFFACL_ERR_HIP);
        if (hipStreamSynchronize(g->engs[i]->home.stream) != hipSuccess) {
            set_last_error("group table broadcast");
            return fail(NFFACL_ERR_HIP);
        }
        table_resident(*g->tabs[i]);
    }
    *out = g;
    return NFFACL_OK;
}

int nffacl_group_size(const nffacl_group *g) { return g ? g->n : NFFACL_ERR_INVALID_ARG; }

int nffacl_group_classify_device(nffacl_group *g, const uint8_t *d_slots, uint32_t stride, uint64_t n,
                                 uint32_t *d_port, uint64_t *d_permit, void *stream) {
    if (!g || (n && !d_slots) || stride < 64 || stride % 16 != 0 || (!d_port && !d_permit) || n > (uint64_t(1) << 48))
        return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    std::lock_guard<std::mutex> lk(g->mu);
    const Rccl &R = rccl();
    hipStream_t rs = static_cast<hipStream_t>(stream);
    std::vector<uint64_t> off(g->n), len(g->n);
    for (int i = 0; i < g->n; ++i) (void)nffacl_group_shard(n, g->n, i, &off[i], &len[i]);
    int st = ensure_staging(g, len[0], stride);  // (the root's shard is the largest)
    if (st != NFFACL_OK) return st;
    int prev = 0;
    (void)hipGetDevice(&prev);
    // scatter: the root's sends to every peer in one group
    if (g->n > 1) {
        CheckedGroup grp(R, "group scatter");
        for (int i = 1; i < g->n && grp.ok(); ++i) {
            if (!len[i]) continue;
            grp.device(g->devs[0]);
            if (grp.ok())
                grp.nccl(R.send(d_slots + off[i] * stride, len[i] * stride, ncclUint8, i, g->comms[0], rs), "ncclSend");
            grp.device(g->devs[i]);
            if (grp.ok()) grp.nccl(R.recv(g->d_in[i], len[i] * stride, ncclUint8, 0, g->comms[i], g->streams[i]), "ncclRecv");
        }
        st = grp.end();
        (void)hipSetDevice(prev);
        if (st != NFFACL_OK) return st;
    }
    // every shard on its own device
    for (int i = 0; i < g->n; ++i) {
        if (!len[i]) continue;
        OnDevice od(g->devs[i]);
        if (!od.ok) return NFFACL_ERR_HIP;
        st = i == 0 ? launch_slots(g->engs[0], g->tabs[0].get(), d_slots, stride, len[0], d_port, d_permit, rs)
                    : launch_slots(g->engs[i], g->tabs[i].get(), g->d_in[i], stride, len[i], d_port ? g->d_out[i] : nullptr,
                                   d_permit ? g->d_perm[i] : nullptr, g->streams[i]);
        if (st != NFFACL_OK) return st;
    }
    // gather the verdicts back into the root's arrays (permit words: off / 64, off is 64-aligned)
    if (g->n > 1) {
        CheckedGroup grp(R, "group gather");
        for (int i = 1; i < g->n && grp.ok(); ++i) {
            if (!len[i]) continue;
            if (d_port) {
                grp.device(g->devs[i]);
                if (grp.ok()) grp.nccl(R.send(g->d_out[i], len[i], ncclUint32, 0, g->comms[i], g->streams[i]), "ncclSend");
                grp.device(g->devs[0]);
                if (grp.ok()) grp.nccl(R.recv(d_port + off[i], len[i], ncclUint32, i, g->comms[0], rs), "ncclRecv");
            }
            if (d_permit) {
                const uint64_t words = (len[i] + 63) / 64;
                grp.device(g->devs[i]);
                if (grp.ok()) grp.nccl(R.send(g->d_perm[i], words, ncclUint64, 0, g->comms[i], g->streams[i]), "ncclSend");
                grp.device(g->devs[0]);
                if (grp.ok()) grp.nccl(R.recv(d_permit + off[i] / 64, words, ncclUint64, i, g->comms[0], rs), "ncclRecv");
            }
        }
        st = grp.end();
        (void)hipSetDevice(prev);
        if (st != NFFACL_OK) return st;
    }
    return NFFACL_OK;
}

void nffacl_group_destroy(nffacl_group *g) {
    if (!g) return;
    group_release(g);
}

}  // extern "C"
