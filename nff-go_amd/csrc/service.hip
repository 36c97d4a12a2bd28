// service.hip — the persistent scalar-call consumer (nffacl_service_*) and the
// per-rule-set device tables (nffacl_rules_prepare) of libnffacl.
//
// Call shape replaced: one packet per call from every flow-function clone —
// pkt.L3ACLPermit(rules) / pkt.L3ACLPort(rules) inside a SetSeparator /
// SetSplitter user function (flow/flow.go:128, 1795-1797;
// examples/firewall/firewall.go:54-57; examples/tutorial/step08.go:33-35),
// with the *L3Rules passed per call and swapped by the user at any time
// (step08.go:38-44).  Layout and protocol: service.hpp.
//
// Device side: one wave64 per kSvcMbPerWave (8) mailboxes, polling with
// sc0 sc1 loads (they bypass L1/L2 and read host memory over PCIe): a wave
// with a mailbox answered in the last `hot` window reads its 1 KiB of
// mailboxes whole with one coalesced load per pass, an idle wave reads only
// its eight bell words.  Complete requests are grouped by
// table generation (wave-uniform descriptor), parsed and classified by the
// same device functions as the batch kernels (classify.hpp), and answered
// with ONE 8-byte system-scope store {tag, port} per request.  The kernel
// leaves after `idle` without requests, after `life` in total, or when the
// host sets the stop word, so every wave reaches its exit on its own.
// Table coherence: a long-lived kernel must not read a table uploaded after
// it started (a DMA write does not reach a stale line of a reused address in
// this XCD's L2; a dispatch invalidates the caches).  Table generations are
// drawn after each upload completes and the armer passes the latest one to
// every launch; a request for a newer table makes every wave leave (ctrl[1])
// and the armer re-launches — once per new table, not per call.
//
// Host side: a caller owns a mailbox (thread-local assignment), writes the
// eight chunks with aligned 16-byte stores (tag chunk last), and spins on its
// response word.  An armer thread launches the kernel when a caller finds it
// not running (a Dekker pair: the caller stores its request and then reads
// `running`; the armer clears `running` after the kernel has exited and then
// re-scans the mailboxes — one of the two always sees the other).
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sched.h>
#include <sys/prctl.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <string>
#include <thread>

#include "classify.hpp"
#include "compile.hpp"
#include "devutil.hpp"
#include "engine.hpp"
#include "rules.hpp"
#include "service.hpp"

#ifndef NFFACL_EXP_SVCSTAT
#define NFFACL_EXP_SVCSTAT 0  // experiment builds (bits): 1 the burst consumer's poll statistic = answer -> next
                              // request; 2 answers without classifying; 4 the stop word read every 64th pass
#endif

namespace nffacl {
namespace dev {

struct SvcArgs {
    const uint8_t *box;     // device alias of the mailboxes (kSvcBoxBytes each), then the bells (u32 each)
    uint64_t *resp;         // device alias of the responses (kSvcRespStride words each)
    uint32_t *ctrl;         // ctrl[0] != 0: stop (host); ctrl[1] != 0: restart (a wave saw a newer table)
    uint32_t box_bytes;     // bytes of the mailbox array (the bells follow it)
    uint32_t range_bytes;   // mailboxes + bells (buffer range)
    uint32_t epoch;         // table generations <= epoch were uploaded before this launch
    uint64_t *stats;        // per wave kSvcStatWords u64 (host memory), written at exit
    uint32_t lds_dwords;    // INDEXED tables up to this size are staged in LDS (0: never)
    uint64_t idle_ticks;    // leave after this long without a request (wall clock ticks)
    uint64_t hot_ticks;     // a mailbox answered within this window is read whole every pass
    uint64_t life_ticks;    // leave after this long in any case
    uint32_t idle_naps;     // burst consumer: s_sleep(8) (~0.2 us) naps of an idle wave between bell reads
    uint32_t post_naps;     // burst consumer: s_sleep(2) (~50 ns) naps after an answer, before the next poll
                            // (the starting value when nap_adapt)
    uint32_t nap_adapt;     // burst consumer: each wave adapts its nap to its caller's turnaround
                            // (NFFACL_TUNE_SVC_POST_NAPS, default 12)
                            // (NFFACL_TUNE_SVC_IDLE_NAPS)
    uint32_t full_poll;     // burst consumer: hot waves read the whole mailbox every pass (default; 0: the
                            // header, then the packets on a new tag — NFFACL_TUNE_SVC_FULLPOLL=0)
};

// One 16-byte chunk of host memory, sc0 sc1 (past L1 and L2: host memory
// written by the CPU is never served stale from a cache).
__device__ __forceinline__ u32x4 ld16_host(__amdgpu_buffer_rsrc_t rs, uint32_t off) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(off), 0, 17));
}

// INDEXED inline entries read from global memory with bounds checks (a word
// outside the table reads as 0 and raises the host flag instead of faulting).
struct CheckedTab {
    static constexpr bool kFreeLoads = false;
    const uint32_t *__restrict__ p;
    uint32_t limit;
    uint32_t *oob;
    __device__ __forceinline__ void flag() const {
        __hip_atomic_store(oob, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __device__ __forceinline__ uint32_t ld(uint32_t i) const {
        if (i < limit) return p[i];
        flag();
        return 0u;
    }
    __device__ __forceinline__ void bounds(uint32_t dir, uint32_t, uint32_t t, uint32_t &lo, uint32_t &hi,
                                           uint32_t = 0) const {
        lo = ld(dir + t);
        hi = ld(dir + t + 1);
    }
    __device__ __forceinline__ u32x4 ld4(uint32_t i) const {
        if (i + 4u <= limit) return reinterpret_cast<const u32x4 *>(p)[i >> 2];
        flag();
        return u32x4{0, 0, 0, 0};
    }
};

// Classify one group (table `tab`, its descriptor `wd` staged in this wave's
// LDS: read where used, so the 80 descriptor words are not held in SGPRs
// across the polling loop).
__device__ __forceinline__ uint32_t svc_classify(const uint32_t *wd, const uint32_t *tab, const Fields &f,
                                                 FlatScratch<2> &W, uint32_t lane, uint32_t *oob, bool staged) {
    // (held in VGPRs until used: readfirstlane'd up front they kept ~80 SGPRs
    // live and spilled; the walks take their per-family values with fam_sel)
    auto w = [&](uint32_t i) -> uint32_t { return wd[i]; };
    const uint32_t kind = __builtin_amdgcn_readfirstlane(wd[0]), ns = __builtin_amdgcn_readfirstlane(wd[1]);
    if (kind == kSvcLinear) return classify_linear(f, tab + w(4), w(5), tab + w(6), w(7));
    IndexedArgs a{};
    a.tab = tab;
    a.dir8 = w(3);
    a.generic = 0;
    a.tab_dwords = w(2);
    a.oob = oob;
    a.live = 0xFFu;
    constexpr uint32_t kFam = 4 + 4 * kMaxSlots;
#pragma unroll
    for (int fam = 0; fam < 2; ++fam) {
        FamArgs &fa = fam ? a.f6 : a.f4;
        const uint32_t b = 8 + kFam * fam;
        fa.off_resid = w(b + 0);
        fa.n_resid = w(b + 1);
        fa.off_cold = w(b + 2);
        fa.off_ent_base = w(b + 3);
#pragma unroll
        for (uint32_t s = 0; s < kMaxSlots; ++s) {
            const uint32_t sh = w(b + 4 + 4 * s);
            fa.slot[s] = SlotArgs{sh & 0xFFu, w(b + 5 + 4 * s), w(b + 6 + 4 * s), w(b + 7 + 4 * s),
                                  s, kFZero, (sh >> 8) & 0xFFu, (sh >> 16) & 0xFFu};
        }
    }
    if (kind == kSvcIndexed && staged) {  // the whole table in LDS (lds_tab[0, tab_dwords))
        if (ns == 2) return classify_indexed<2, 1>(LdsTab{}, a, f);
        if (ns == 3) return classify_indexed<3, 1>(LdsTab{}, a, f);
        return classify_indexed<4, 1>(LdsTab{}, a, f);
    }
    if (kind == kSvcIndexed) {
        const CheckedTab ct{tab, a.tab_dwords, oob};
        if (ns == 2) return classify_indexed<2, 1>(ct, a, f);
        if (ns == 3) return classify_indexed<3, 1>(ct, a, f);
        return classify_indexed<4, 1>(ct, a, f);
    }
    if (kind == kSvcFlat) {
        if (ns == 2) return classify_flat<2, 2, true, false, false>(a, f, W, lane);
        if (ns == 3) return classify_flat<3, 2, true, false, false>(a, f, W, lane);
        if (ns == 4) return classify_flat<4, 2, true, false, false>(a, f, W, lane);
        if (ns == 5) return classify_flat<5, 2, true, false, false>(a, f, W, lane);
        if (ns == 6) return classify_flat<6, 2, true, false, false>(a, f, W, lane);
        if (ns == 7) return classify_flat<7, 2, true, false, false>(a, f, W, lane);
        return classify_flat<8, 2, true, false, false>(a, f, W, lane);
    }
    return 0u;
}

__global__ void __launch_bounds__(64) k_service(SvcArgs a) {
    __shared__ FlatScratch<2> W;
    const uint32_t lane = lane_id();
    constexpr uint32_t MPW = kSvcMbPerWave;
    const bool has_mb = lane < MPW;  // lanes 0..MPW-1 own the wave's mailboxes
    const uint32_t mb = blockIdx.x * MPW + (has_mb ? lane : 0u);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.box), 0,
                                                                        static_cast<int>(a.range_bytes), 0x00020000);
    uint64_t *resp = a.resp + size_t(mb) * kSvcRespStride;
    uint32_t done = 0;
    if (has_mb) done = static_cast<uint32_t>(__hip_atomic_load(resp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> 32);
    const uint64_t t0 = wall_clock64();
    uint64_t last = t0, lane_last = t0;  // hot at start: the call that armed us is read whole
    uint32_t cur_key = 0xFFFFFFFFu;  // generation << 1 | vlan of the descriptor in `w`
    uint32_t staged_gen = 0xFFFFFFFFu;  // generation of the table staged in LDS
    __shared__ __attribute__((aligned(16))) uint32_t wd[kSvcDescDwords];  // the current table's descriptor
    uint32_t w_kind = 0, w_dwords = 0;  // its kind and table size (wave-uniform)
    const uint32_t *tab = nullptr;
    // where the time goes (wall-clock ticks, written to host memory at exit):
    // polls and their ticks (issue to data), groups classified and their
    // ticks, requests answered
    uint64_t n_polls = 0, poll_ticks = 0, n_groups = 0, group_ticks = 0, n_req = 0;
    // One poll always in flight: the next pass's mailbox reads are issued as
    // soon as this pass's data is in registers, before its requests are
    // classified, so the PCIe round trip overlaps the classification
    // (LDS-staged tables issue no vector memory reads that would wait behind
    // it).  A poll reads the whole mailbox of lanes answered within `hot`,
    // only the tag chunk of the others.
    // A wave owns MPW mailboxes.  While one of them is hot the wave reads all
    // of them whole, each load instruction 1 KiB contiguous (lane l: bytes
    // 16 l of that KiB, i.e. chunk l % 8 of mailbox l / 8) — a few large PCIe
    // reads instead of a 16-byte read per chunk per lane — and hands each
    // mailbox lane its own eight chunks through LDS; an idle wave reads only
    // its MPW bells (contiguous u32s).  Small waves keep every poll one
    // round trip short and let the waves of busy mailboxes classify in
    // parallel on their own SIMDs.
    constexpr uint32_t kLoads = MPW * kSvcBoxBytes / 1024u;
    __shared__ u32x4 img[64 * kLoads];
    const uint32_t wave_box = blockIdx.x * MPW * kSvcBoxBytes;
    const uint32_t bell = a.box_bytes + mb * 4u;
    u32x4 nx[kLoads];
    uint32_t nbell = 0;
    uint64_t ncw = 0, nt = t0;
    bool nhot = true;
    // (round 4: the burst consumer's order — stop word first by every lane,
    // bells unconditionally — ran 5.20 / 5.35 vs 5.86 / 5.63 Mpps at 32
    // threads here, profiles/r4_service/scalar_poll_order/: not kept)
    auto issue = [&]() {
        nt = wall_clock64();
        nhot = ballot(has_mb && nt - lane_last <= a.hot_ticks) != 0u;  // wave-uniform
#pragma unroll
        for (uint32_t j = 0; j < kLoads; ++j) nx[j] = u32x4{0, 0, 0, 0};
        nbell = 0;
        if (nhot) {
#pragma unroll
            for (uint32_t j = 0; j < kLoads; ++j) nx[j] = ld16_host(rs, wave_box + 1024u * j + 16u * lane);
        } else if (has_mb) {
            nbell = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(bell), 0, 17);
        }
        ncw = 0;  // stop | restart << 32
        if (lane == 0) ncw = __hip_atomic_load(reinterpret_cast<uint64_t *>(a.ctrl), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
    };
    issue();
    while (true) {
        u32x4 c[kSvcChunks];
        const uint64_t cw = ncw, now = nt;
        const bool hot = nhot;
#pragma unroll
        for (uint32_t j = 0; j < kSvcChunks; ++j) c[j] = u32x4{0, 0, 0, 0};
        if (hot) {  // the poll issued a pass ago: every mailbox lane its own chunks, through LDS
#pragma unroll
            for (uint32_t j = 0; j < kLoads; ++j) img[64u * j + lane] = nx[j];
            wave_lds_sync();
            if (has_mb) {
#pragma unroll
                for (uint32_t j = 0; j < kSvcChunks; ++j) c[j] = img[kSvcChunks * lane + j];
            }
            wave_lds_sync();
        } else {
            c[kSvcChunks - 1].w = nbell;
        }
        if (now - t0 > a.life_ticks) break;
        issue();  // the next pass's poll, in flight from here
        if ((__builtin_amdgcn_readlane(static_cast<uint32_t>(cw), 0) |
             __builtin_amdgcn_readlane(static_cast<uint32_t>(cw >> 32), 0)) != 0u)
            break;
        const uint32_t tag = c[kSvcChunks - 1].w;
        const bool fresh = has_mb && tag != done;
        const uint64_t t_data = wall_clock64();
        ++n_polls;
        poll_ticks += t_data - now;
        // a new tag on a bell turns the wave hot: mailboxes read whole from the poll after next
        if (!hot && fresh) lane_last = now;
        bool pend = hot && fresh;
#pragma unroll
        for (uint32_t j = 0; j + 1 < kSvcChunks; ++j) pend = pend && c[j].w == tag;  // untorn
        uint64_t m = ballot(pend);
        if (!ballot(fresh)) {
            if (now - last > a.idle_ticks) break;
            continue;
        }
        last = now;
        bool restart = false;
        while (m) {
            const uint64_t t_group = wall_clock64();
            const uint32_t first = static_cast<uint32_t>(__builtin_ctzll(m));
            const uint32_t key = __builtin_amdgcn_readlane(c[kSvcChunks - 1].z, first);
            const bool mine = pend && c[kSvcChunks - 1].z == key;
            if (key == kSvcWithdrawn) {  // the caller gave up: answered, no table read
                if (mine) {
                    __hip_atomic_store(resp, uint64_t(tag) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    done = tag;
                }
                pend = pend && !mine;
                m = ballot(pend);
                continue;
            }
            if ((key >> 1) > a.epoch) {
                // a table uploaded after this launch: its bytes are visible to
                // a NEW launch (the dispatch invalidates the caches), not
                // necessarily to this one (a reused address can still sit in
                // this XCD's L2).  Every wave leaves; the armer re-launches.
                if (lane == 0) __hip_atomic_store(a.ctrl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                restart = true;
                break;
            }
            if (key != cur_key) {
                // the descriptor of a table this wave has not walked yet (all
                // its loads in flight together; the table predates this
                // launch, so no cache level can hold an older copy of it)
                // (readlane returns int: through uint32_t, or the low word sign-extends)
                const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(c[kSvcChunks - 1].x, first));
                const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(c[kSvcChunks - 1].y, first));
                const u32x4 *dq = reinterpret_cast<const u32x4 *>(hi << 32 | lo);
                if (lane < kSvcDescDwords / 4) reinterpret_cast<u32x4 *>(wd)[lane] = dq[lane];
                wave_lds_sync();
                w_kind = __builtin_amdgcn_readfirstlane(wd[0]);
                w_dwords = __builtin_amdgcn_readfirstlane(wd[2]);
                tab = reinterpret_cast<const uint32_t *>(hi << 32 | lo) - w_dwords;
                cur_key = key;
            }
            // small INDEXED tables are walked from LDS: staged once per table
            // (per launch), and then no table read waits behind the PCIe polls
            const bool staged = w_kind == kSvcIndexed && w_dwords <= a.lds_dwords;
            if (staged && staged_gen != (key >> 1)) {
                const u32x4 *src = reinterpret_cast<const u32x4 *>(tab);
                u32x4 *dst = reinterpret_cast<u32x4 *>(lds_tab);
                for (uint32_t i = lane; i < (w_dwords + 3u) / 4u; i += 64u) dst[i] = src[i];
                wave_lds_sync();
                staged_gen = key >> 1;
            }
            uint32_t full[3 * kSvcPktChunks], d[16];
#pragma unroll
            for (uint32_t j = 0; j < kSvcPktChunks; ++j) {
                full[3 * j + 0] = c[j].x;
                full[3 * j + 1] = c[j].y;
                full[3 * j + 2] = c[j].z;
            }
#pragma unroll
            for (int k = 0; k < 16; ++k) d[k] = full[k];
            Fields f;
            parse_fields<true>(d, mine, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
                lo = 0;
                hi = 0;
#pragma unroll
                for (uint32_t j = 0; j < 3 * kSvcPktChunks; ++j) {
                    lo = k == j ? full[j] : lo;
                    hi = k + 1 == j ? full[j] : hi;
                }
            }, key & 1u ? uint32_t(NFFACL_PARSE_VLAN) : 0u);
            const uint32_t port = svc_classify(wd, tab, f, W, lane, a.ctrl + 2, staged);
            if (mine) {
                __hip_atomic_store(resp, uint64_t(tag) << 32 | port, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                done = tag;
                lane_last = now;
            }
            pend = pend && !mine;
            m = ballot(pend);
            ++n_groups;
            n_req += __builtin_popcountll(ballot(mine));
            group_ticks += wall_clock64() - t_group;
        }
        if (restart) break;
    }
    if (lane == 0) {
        uint64_t *st = a.stats + size_t(blockIdx.x) * kSvcStatWords;
        const uint64_t v[5] = {n_polls, poll_ticks, n_groups, group_ticks, n_req};
#pragma unroll
        for (int i = 0; i < 5; ++i) __hip_atomic_store(st + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The burst consumer: one wave per burst mailbox (service.hpp), lane i
// classifies packet i of the mailbox's request.  A hot wave (answered within
// `hot`) reads its whole mailbox (3.6 KB, four 1 KiB loads) once per pass and
// issues the next pass's poll only after answering: a poll issued before the
// answer is out can never hold the caller's next request, it only loads the
// PCIe link.  An idle wave reads only its bell word.  (Round 4, C2 rules,
// 16 / 32 clones: polls issued a pass ahead 55 / 103 Mpps; header-only polls
// + one read of the packets per request (full_poll = 0,
// NFFACL_TUNE_SVC_FULLPOLL=0) 56 / 103; whole-mailbox polls issued after
// the answer 67 / 132 — profiles/r4_service/.)  A request is one rule set:
// no grouping, the descriptor is wave-uniform.
// Longest adaptive post-answer nap (s_sleep 2 units, ~50 ns each: ~2 us).
constexpr uint32_t kSvcNapMax = 40;

__global__ void __launch_bounds__(64) k_service_burst(SvcArgs a) {
    __shared__ FlatScratch<2> W;
    __shared__ u32x4 img[64 * kSvcBurstLoads];
    const uint32_t lane = lane_id();
    const uint32_t mb = blockIdx.x;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(a.box), 0,
                                                                        static_cast<int>(a.range_bytes), 0x00020000);
    uint64_t *resp = a.resp + size_t(mb) * kSvcBurstRespWords;
    // the last tag answered: every answer writes word 0 (n >= 1)
    uint32_t done = __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(__hip_atomic_load(resp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> 32));
    const uint64_t t0 = wall_clock64();
    uint64_t last = t0, ans_last = t0;  // hot at start: the call that armed us is read whole
    uint32_t cur_key = 0xFFFFFFFFu, staged_gen = 0xFFFFFFFFu;
    __shared__ __attribute__((aligned(16))) uint32_t wd[kSvcDescDwords];  // the current table's descriptor
    uint32_t w_kind = 0, w_dwords = 0;  // its kind and table size (wave-uniform)
    const uint32_t *tab = nullptr;
    uint64_t n_polls = 0, poll_ticks = 0, n_groups = 0, group_ticks = 0, n_req = 0, n_torn = 0;
#if NFFACL_EXP_SVCSTAT
    uint64_t t_ans = 0;
#endif
    const uint32_t box = mb * kSvcBurstBoxBytes;
    const uint32_t bell = a.box_bytes + mb * 4u;
    uint32_t nap = a.post_naps;  // the post-answer nap (wave-uniform; adapted when a.nap_adapt)
    bool answered = false;       // this pass's poll is the first after an answer
    while (true) {
        // one poll per pass, issued here (see above)
        const uint64_t now = wall_clock64();
        if (now - t0 > a.life_ticks) break;
        const bool hot = now - ans_last <= a.hot_ticks;  // wave-uniform
        // Every read of the pass is issued before the first wait: the stop
        // word (all lanes: one coalesced request), then the whole mailbox
        // (all lanes, all four loads: the last KiB past a full request is
        // read and ignored), or the header / the bell.  (Round 4: with the
        // tail load under a lane mask and the stop word read by lane 0 after
        // it, the compiler waited for the first three loads before issuing
        // them — two PCIe round trips per pass.)
        const uint64_t cw = (NFFACL_EXP_SVCSTAT & 4) && (n_polls & 63u) != 0u  // (experiment 4: every 64th pass)
                                ? 0ull
                                : __hip_atomic_load(reinterpret_cast<uint64_t *>(a.ctrl), __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_SYSTEM);  // stop | restart << 32
        u32x4 body[kSvcBurstLoads];
        u32x4 hh;  // lane 0 chunk 0, lane 1 chunk 1
        uint32_t bl = 0;
        if (hot && a.full_poll) {
#pragma unroll
            for (uint32_t j = 0; j < kSvcBurstLoads; ++j) body[j] = ld16_host(rs, box + 1024u * j + 16u * lane);
            hh = body[0];
        } else {
#pragma unroll
            for (uint32_t j = 0; j < kSvcBurstLoads; ++j) body[j] = u32x4{0, 0, 0, 0};
            hh = u32x4{0, 0, 0, 0};
            if (hot) {
                if (lane < kSvcBurstHdrChunks) hh = ld16_host(rs, box + 16u * lane);
            } else if (lane == 0) {
                bl = __builtin_amdgcn_raw_buffer_load_b32(rs, static_cast<int>(bell), 0, 17);
            }
        }
        const uint32_t tag = hot ? static_cast<uint32_t>(__builtin_amdgcn_readlane(hh.w, 0))
                                 : static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(bl));
        if ((__builtin_amdgcn_readlane(static_cast<uint32_t>(cw), 0) |
             __builtin_amdgcn_readlane(static_cast<uint32_t>(cw >> 32), 0)) != 0u)
            break;
        const uint64_t t_data = wall_clock64();
#if !(NFFACL_EXP_SVCSTAT & 1)
        ++n_polls;
        poll_ticks += t_data - now;
#endif
        if (tag == done) {
            // the first poll after an answer came back empty: the caller had
            // not posted yet, and its request now waits a whole extra round
            // trip — nap longer after the next answer
            if (answered && a.nap_adapt) nap = min(nap + 3u, kSvcNapMax);
            answered = false;
            if (now - last > a.idle_ticks) break;
            // an idle wave naps between bell reads (its reads share the
            // link's request slots with the hot waves' polls)
            if (!hot)
                for (uint32_t i = 0; i < a.idle_naps; ++i) __builtin_amdgcn_s_sleep(8);
            continue;
        }
        last = now;
        if (!hot) {  // a new tag on the bell: the next pass polls the header
            ans_last = now;
            continue;
        }
        // header complete (both chunks carry the tag): read the packets' chunks
        const uint32_t n = __builtin_amdgcn_readlane(hh.x, 1);
        if (static_cast<uint32_t>(__builtin_amdgcn_readlane(hh.w, 1)) != tag || n == 0u || n > kSvcBurstMax) {
            ++n_torn;  // raced the host's stores: the next poll has it
            continue;
        }
#if NFFACL_EXP_SVCSTAT & 8  // experiment: answer at once (no packet read, transposition or classification)
        if (lane < n) __hip_atomic_store(resp + lane, uint64_t(tag) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        done = tag;
        ans_last = now;
        ++n_groups;
        n_req += n;
#if NFFACL_EXP_SVCSTAT & 1
        if (t_ans) {
            ++n_polls;
            poll_ticks += t_data - t_ans;
        }
        t_ans = wall_clock64();
#endif
        continue;
#endif
        if (!a.full_poll) {
            const uint32_t nl = ((kSvcBurstHdrChunks + kSvcBurstPktChunks * n) * 16u + 1023u) / 1024u;  // 1 KiB loads
#pragma unroll
            for (uint32_t j = 0; j < kSvcBurstLoads; ++j)
                body[j] = j < nl ? ld16_host(rs, box + 1024u * j + 16u * lane) : u32x4{0, 0, 0, 0};
        }
        // through LDS: lane i gets packet i's chunks
#pragma unroll
        for (uint32_t j = 0; j < kSvcBurstLoads; ++j) img[64u * j + lane] = body[j];
        wave_lds_sync();
        u32x4 c[kSvcBurstPktChunks];
#pragma unroll
        for (uint32_t j = 0; j < kSvcBurstPktChunks; ++j)
            c[j] = lane < kSvcBurstMax ? img[kSvcBurstHdrChunks + kSvcBurstPktChunks * lane + j] : u32x4{0, 0, 0, 0};
        wave_lds_sync();
        // complete when every chunk of packets 0..n-1 carries the tag
        const bool live = lane < n;
        bool torn = false;
#pragma unroll
        for (uint32_t j = 0; j < kSvcBurstPktChunks; ++j) torn = torn || (live && c[j].w != tag);
        if (ballot(torn)) {  // the packets' stores not all visible yet: the next poll re-reads them
            ++n_torn;
            continue;
        }
        // found on the first poll after the answer: probe a shorter nap
        if (answered && a.nap_adapt && nap > 0u) --nap;
        answered = false;
        u32x4 h0;
        h0.x = __builtin_amdgcn_readlane(hh.x, 0);
        h0.y = __builtin_amdgcn_readlane(hh.y, 0);
        h0.z = __builtin_amdgcn_readlane(hh.z, 0);
        const uint64_t t_group = wall_clock64();
#if NFFACL_EXP_SVCSTAT & 1  // experiment: "polls" = answer -> next request seen, per hot wave
        if (t_ans) {
            ++n_polls;
            poll_ticks += t_data - t_ans;
        }
#endif
        const uint32_t key = __builtin_amdgcn_readfirstlane(h0.z);
        if (key == kSvcWithdrawn) {  // the caller gave up: answered, no table read
            if (live) __hip_atomic_store(resp + lane, uint64_t(tag) << 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            done = tag;
            continue;
        }
        if ((key >> 1) > a.epoch) {  // a table uploaded after this launch (see k_service)
            if (lane == 0) __hip_atomic_store(a.ctrl + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        if (key != cur_key) {
            // (readfirstlane returns int: through uint32_t, or the low word sign-extends)
            const uint64_t lo = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(h0.x));
            const uint64_t hi = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(h0.y));
            const u32x4 *dq = reinterpret_cast<const u32x4 *>(hi << 32 | lo);
            if (lane < kSvcDescDwords / 4) reinterpret_cast<u32x4 *>(wd)[lane] = dq[lane];
            wave_lds_sync();
            w_kind = __builtin_amdgcn_readfirstlane(wd[0]);
            w_dwords = __builtin_amdgcn_readfirstlane(wd[2]);
            tab = reinterpret_cast<const uint32_t *>(hi << 32 | lo) - w_dwords;
            cur_key = key;
        }
        const bool staged = w_kind == kSvcIndexed && w_dwords <= a.lds_dwords;
        if (staged && staged_gen != (key >> 1)) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(tab);
            u32x4 *dst = reinterpret_cast<u32x4 *>(lds_tab);
            for (uint32_t i = lane; i < (w_dwords + 3u) / 4u; i += 64u) dst[i] = src[i];
            wave_lds_sync();
            staged_gen = key >> 1;
        }
        // bytes 0..83 of the packet: the MAC addresses (0-11) were not sent
        uint32_t full[3 * kSvcPktChunks], d[16];
        full[0] = full[1] = full[2] = 0u;
#pragma unroll
        for (uint32_t j = 0; j < kSvcBurstPktChunks; ++j) {
            full[3 * j + 3] = c[j].x;
            full[3 * j + 4] = c[j].y;
            full[3 * j + 5] = c[j].z;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) d[k] = full[k];
        Fields f;
        parse_fields<true>(d, live, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
            lo = 0;
            hi = 0;
#pragma unroll
            for (uint32_t j = 0; j < 3 * kSvcPktChunks; ++j) {
                lo = k == j ? full[j] : lo;
                hi = k + 1 == j ? full[j] : hi;
            }
        }, key & 1u ? uint32_t(NFFACL_PARSE_VLAN) : 0u);
#if NFFACL_EXP_SVCSTAT & 2  // experiment: answer without classifying (verdicts wrong)
        const uint32_t port = f.proto;
#else
        const uint32_t port = svc_classify(wd, tab, f, W, lane, a.ctrl + 2, staged);
#endif
        if (live) __hip_atomic_store(resp + lane, uint64_t(tag) << 32 | port, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        done = tag;
        ans_last = now;
        ++n_groups;
        n_req += n;
        group_ticks += wall_clock64() - t_group;
#if NFFACL_EXP_SVCSTAT
        t_ans = wall_clock64();
#endif
        // Wait ~0.6 us before the next poll: one issued at once reaches the
        // mailbox before the caller has seen this answer and posted its next
        // burst, returns empty, and the request waits for the poll after it —
        // a whole PCIe round trip.  C2 rules, 16 / 32 clones: 87-103 /
        // 147-160 Mpps without the nap, 122-124 / 182-191 with 12 naps (6 / 8
        // / 10 / 15: 97-102 / 100-112 / 107-119 / 120-121 at 16 clones;
        // NFFACL_TUNE_SVC_POST_NAPS, profiles/r5_ab/burst/)
        // Round 6: each wave adapts the nap to its own caller (nap_adapt):
        // +3 after an empty first poll (a whole PCIe round trip lost), -1
        // after a first poll that found the request — it settles just past
        // the caller's turnaround, whichever host it runs on.
        for (uint32_t i = 0; i < nap; ++i) __builtin_amdgcn_s_sleep(2);
        answered = true;
    }
    if (lane == 0) {
        uint64_t *st = a.stats + size_t(blockIdx.x) * kSvcStatWords;
        const uint64_t v[6] = {n_polls, poll_ticks, n_groups, group_ticks, n_req, n_torn};
#pragma unroll
        for (int i = 0; i < 6; ++i) __hip_atomic_store(st + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace dev

// ---- per-rule-set device tables -----------------------------------------------

namespace {

// One table home per device for the rule-set tables (uploads + stream-ordered
// retirement), created on first use and kept for the life of the process.
TableHome *rules_home(int dev) {
    static std::once_flag once[kMaxDevices];
    static TableHome *homes[kMaxDevices];
    std::call_once(once[dev], [dev] {
        auto *h = new TableHome();
        if (h->init(dev) != hipSuccess) {
            (void)hipGetLastError();
            delete h;
            h = nullptr;
        }
        homes[dev] = h;
    });
    return homes[dev];
}

struct DeviceRestore {
    int old = -1;
    explicit DeviceRestore(int dev) {
        if (hipGetDevice(&old) != hipSuccess) old = -1;
        if (old != dev) (void)hipSetDevice(dev);
    }
    ~DeviceRestore() {
        if (old >= 0) (void)hipSetDevice(old);
    }
};

}  // namespace

DevTable *rules_table(const nffacl_rules *r, int dev, int &st) {
    st = NFFACL_OK;
    if (!r || dev < 0 || dev >= kMaxDevices) {
        st = NFFACL_ERR_INVALID_ARG;
        return nullptr;
    }
    DevTable *t = r->dev[dev].load(std::memory_order_acquire);
    if (t) return t;
    std::lock_guard<std::mutex> g(r->dev_mu);
    t = r->dev[dev].load(std::memory_order_relaxed);
    if (t) return t;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_last_error("no HIP device visible");
        st = NFFACL_ERR_NO_DEVICE;
        return nullptr;
    }
    if (dev >= count) {
        st = NFFACL_ERR_INVALID_ARG;
        return nullptr;
    }
    DeviceRestore ds(dev);
    if ((st = prepare_kernels()) != NFFACL_OK) return nullptr;
    TableHome *home = rules_home(dev);
    if (!home) {
        set_last_error("rules table home: stream creation failed");
        st = NFFACL_ERR_HIP;
        return nullptr;
    }
    home->reap(false);
    // default layout (no tuning knobs): the forms the scalar consumer walks
    auto *nt = new (std::nothrow) DevTable();
    if (!nt) {
        st = NFFACL_ERR_NOMEM;
        return nullptr;
    }
    st = compile_upload(*r, NFFACL_ALGO_AUTO, CompileOptions{}, *home, *nt);
    if (st != NFFACL_OK) {
        delete nt;
        return nullptr;
    }
    r->dev[dev].store(nt, std::memory_order_release);
    return nt;
}

void release_rules_tables(const nffacl_rules *r) {
    for (int dev = 0; dev < kMaxDevices; ++dev) {
        DevTable *t = r->dev[dev].exchange(nullptr, std::memory_order_acq_rel);
        if (!t) continue;
        delete t;  // retires stream-ordered behind the batch launches that used it (tables.hpp)
        if (TableHome *h = rules_home(dev)) h->reap(false);
    }
}

}  // namespace nffacl

// ---- the service object ---------------------------------------------------------

using namespace nffacl;
using Clock = std::chrono::steady_clock;

namespace {

struct alignas(64) MailboxState {
    std::atomic<uint32_t> lock{0};  // owner (threads beyond the mailbox count share)
    uint32_t seq = 0;               // last tag posted
    uint32_t nap = 0;               // under lock: this mailbox's adaptive nap after posting, ns
};

// CPUs this process may keep busy: its affinity mask, capped by a cgroup v2
// CPU quota ("QUOTA PERIOD" in cpu.max) when one is set.
uint32_t cpu_budget() {
    cpu_set_t set;
    uint32_t n = 0;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = static_cast<uint32_t>(CPU_COUNT(&set));
    if (n == 0) n = std::max(1u, std::thread::hardware_concurrency());
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long period = 0;
        if (std::fscanf(f, "%31s %lu", q, &period) == 2 && period > 0 && std::isdigit(static_cast<unsigned char>(q[0])))
            n = std::min<uint32_t>(n, std::max(1ul, (std::strtoul(q, nullptr, 10) + period - 1) / period));
        std::fclose(f);
    }
    return n;
}

}  // namespace

struct nffacl_service {
    // NFFACL_TUNE_SVC_TRACE=1 (experiments): host-side phase times of the
    // calls, printed to stderr when the service is destroyed
    bool trace = false;
    std::atomic<uint64_t> tr_calls{0}, tr_total_ns{0}, tr_post_ns{0}, tr_wait_ns{0}, tr_spins{0};
    int device = 0;
    uint32_t id = 0;  // process-unique: keys the callers' thread-local mailbox choice
    uint32_t n_mb = 0;
    // burst service (nffacl_service_create_burst): burst mailboxes, one
    // consumer wave each (k_service_burst); else scalar mailboxes, 8 per wave
    bool burst = false;
    uint32_t box_stride = kSvcBoxBytes;       // bytes per mailbox
    uint32_t resp_stride = kSvcRespStride;    // u64 response words per mailbox
    // a call waits this long for its answer, re-posts once, waits again, and
    // then withdraws its request (NFFACL_TUNE_SVC_TIMEOUT_US)
    uint64_t timeout_us = 1000000;
    // After posting, a caller sleeps through most of the round trip instead
    // of spinning it once the callers outnumber the CPUs this process may use
    // (sleep_ns < 0: adaptive, per mailbox; 0: never; > 0: fixed;
    // NFFACL_TUNE_SVC_SLEEP_NS).  Under a CPU quota every spinning caller
    // burns the quota the others need: throughput = quota / CPU per call.
    int32_t sleep_ns = -1;
    uint32_t cpus = 1;
    // requests written with non-temporal (streaming) stores + sfence: the
    // lines go to memory, not into the writing core's cache, so the GPU's
    // snooped PCIe reads of them need no cache-to-IO transfer
    // (NFFACL_TUNE_SVC_NT)
    bool nt = false;
    uint8_t *h_mem = nullptr;  // mapped, coherent pinned host memory: boxes | responses | ctrl
    uint8_t *h_box = nullptr;
    uint32_t *h_bell = nullptr;   // per mailbox: the tag of its latest request (written after the chunks)
    uint64_t *h_resp = nullptr;
    uint32_t *h_ctrl = nullptr;
    uint64_t *h_stats = nullptr;  // per wave: the consumer's counters of its last launch
    uint64_t acc[kSvcStatWords] = {};  // under mu: summed over launches
    uint64_t ticks_per_us = 100;
    dev::SvcArgs args{};
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    std::unique_ptr<MailboxState[]> mbx;
    std::atomic<uint32_t> next_mb{0};
    std::atomic<bool> running{false};
    std::atomic<int> error{NFFACL_OK};
    std::string error_msg;  // under mu: what failed in the armer thread
    std::mutex mu;
    std::condition_variable cv;
    bool kick = false, stop = false;
    std::thread armer;
    std::atomic<uint64_t> launches{0}, requests{0}, timeouts{0}, retries{0};
    std::atomic<bool> paused{false};  // nffacl_service_pause: no consumer launches
    uint32_t waves() const { return burst ? n_mb : n_mb / kSvcMbPerWave; }
};

namespace {

// Live services, stopped at process exit (a kernel still polling host memory
// that the exiting process unmaps would fault).
std::mutex g_live_mu;
std::set<nffacl_service *> *g_live = nullptr;
std::atomic<uint32_t> g_next_id{1};

void stop_kernel(nffacl_service *s) {
    __atomic_store_n(s->h_ctrl, 1u, __ATOMIC_RELEASE);
    {
        std::lock_guard<std::mutex> g(s->mu);
        s->stop = true;
    }
    s->cv.notify_all();
    if (s->armer.joinable()) s->armer.join();
}

void stop_all_at_exit() {
    std::lock_guard<std::mutex> g(g_live_mu);
    if (!g_live) return;
    for (nffacl_service *s : *g_live) stop_kernel(s);
}

// the tag of a mailbox's latest request (scalar: chunk 7, burst: chunk 0)
uint32_t box_tag(const nffacl_service *s, uint32_t i) {
    const size_t at = size_t(i) * s->box_stride + (s->burst ? 12 : kSvcBoxBytes - 4);
    return __atomic_load_n(reinterpret_cast<const uint32_t *>(s->h_box + at), __ATOMIC_ACQUIRE);
}

uint32_t resp_tag(const nffacl_service *s, uint32_t i) {
    return static_cast<uint32_t>(__atomic_load_n(s->h_resp + size_t(i) * s->resp_stride, __ATOMIC_ACQUIRE) >> 32);
}

bool any_pending(const nffacl_service *s) {
    for (uint32_t i = 0; i < s->n_mb; ++i)
        if (box_tag(s, i) != resp_tag(s, i)) return true;
    return false;
}

void armer_main(nffacl_service *s) {
    (void)hipSetDevice(s->device);
    (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);  // its naps: 20 us, not 20 + 50 us
    std::unique_lock<std::mutex> lk(s->mu);
    while (true) {
        s->cv.wait(lk, [&] { return s->kick || s->stop; });
        if (s->stop) break;
        s->kick = false;
        if (s->paused.load(std::memory_order_acquire)) continue;  // nffacl_service_pause: re-armed by the resume
        lk.unlock();
        s->running.store(true, std::memory_order_seq_cst);
        __atomic_store_n(&s->h_ctrl[1], 0u, __ATOMIC_SEQ_CST);
        s->args.epoch = table_epoch();  // every table of this generation or older is in HBM
        s->launches.fetch_add(1, std::memory_order_relaxed);  // (before the launch: its calls may return first)
        if (s->burst)
            hipLaunchKernelGGL(dev::k_service_burst, dim3(s->waves()), dim3(64), size_t(s->args.lds_dwords) * 4,
                               s->stream, s->args);
        else
            hipLaunchKernelGGL(dev::k_service, dim3(s->waves()), dim3(64), size_t(s->args.lds_dwords) * 4,
                               s->stream, s->args);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(s->done, s->stream);
        if (e == hipSuccess) {
            // Sleep-poll for the kernel's exit: a blocking hipEventSynchronize
            // still kept one CPU busy for the kernel's whole life (round 3 sweep:
            // 2.0 CPUs at one caller), and under a CPU quota that CPU is the
            // callers'.  20 us late at most, once per launch.
            const timespec nap{0, 20000};
            while ((e = hipEventQuery(s->done)) == hipErrorNotReady) (void)nanosleep(&nap, nullptr);
        }
        s->running.store(false, std::memory_order_seq_cst);
        lk.lock();
        for (uint32_t wv = 0; wv < s->waves(); ++wv)
            for (uint32_t i = 0; i < kSvcStatWords; ++i) {
                s->acc[i] += __atomic_load_n(&s->h_stats[wv * kSvcStatWords + i], __ATOMIC_ACQUIRE);
                __atomic_store_n(&s->h_stats[wv * kSvcStatWords + i], 0ull, __ATOMIC_RELAXED);
            }
        if (e != hipSuccess) {
            s->error_msg = std::string("service consumer: ") + hipGetErrorName(e) + ": " + hipGetErrorString(e);
            s->error.store(NFFACL_ERR_HIP, std::memory_order_release);
        }
        // a request posted after the kernel's last poll: launch again at once
        if (e == hipSuccess && any_pending(s)) s->kick = true;
    }
}

void kick(nffacl_service *s) {
    {
        std::lock_guard<std::mutex> g(s->mu);
        s->kick = true;
    }
    s->cv.notify_one();
}

// This thread's mailbox of service `s` (assigned on first use, round robin).
uint32_t my_mailbox(nffacl_service *s) {
    struct Slot {
        uint32_t id = 0, mb = 0;
    };
    thread_local Slot cache[4];
    thread_local uint32_t victim = 0;
    for (Slot &c : cache)
        if (c.id == s->id) return c.mb;
    Slot &c = cache[victim++ % 4];
    c.id = s->id;
    // consecutive threads on different waves: each wave polls and classifies
    // for few callers, the waves of busy mailboxes in parallel
    const uint32_t k = s->next_mb.fetch_add(1, std::memory_order_relaxed) % s->n_mb;
    const uint32_t waves = s->waves();
    c.mb = s->burst ? k : (k % waves) * kSvcMbPerWave + k / waves;
    return c.mb;
}

void release_service(nffacl_service *s) {
    if (s->trace && s->tr_calls.load()) {
        const double c = double(s->tr_calls.load());
        std::fprintf(stderr, "[nffacl service trace] calls %.0f: total %.3f us, post %.3f us, wait %.3f us, spins %.1f per call\n",
                     c, s->tr_total_ns.load() / c / 1e3, s->tr_post_ns.load() / c / 1e3, s->tr_wait_ns.load() / c / 1e3,
                     s->tr_spins.load() / c);
    }
    if (s->done) (void)hipEventDestroy(s->done);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->h_mem) (void)hipHostFree(s->h_mem);
    delete s;
}

}  // namespace

namespace {

// NUMA node of every HIP device (from its PCI function's sysfs entry), read once.
struct DeviceNodes {
    int count = 0;
    int node[kMaxDevices];
};

const DeviceNodes &device_nodes() {
    static DeviceNodes dn;
    static std::once_flag once;
    std::call_once(once, [] {
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess) {
            (void)hipGetLastError();
            count = 0;
        }
        dn.count = std::min(count, kMaxDevices);
        for (int d = 0; d < dn.count; ++d) {
            dn.node[d] = -1;
            char bus[64] = {0};
            if (hipDeviceGetPCIBusId(bus, sizeof bus, d) != hipSuccess) {
                (void)hipGetLastError();
                continue;
            }
            for (char *c = bus; *c; ++c) *c = static_cast<char>(std::tolower(static_cast<unsigned char>(*c)));
            const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
            if (FILE *f = std::fopen(path.c_str(), "r")) {
                int n = -1;
                if (std::fscanf(f, "%d", &n) == 1) dn.node[d] = n;
                std::fclose(f);
            }
        }
    });
    return dn;
}

// Pinned host memory on NUMA node `node` (< 0: wherever the calling thread
// allocates).  The mailboxes are read by the GPU over PCIe and spun on by the
// callers: on the node of the GPU's PCIe root the consumer's poll round trip
// is 2.0 us and one request's classification 1.1 us; on the other socket 2.9
// and 1.9 us (32 callers: 5.9 vs 3.9 Mpps, profiles/r3_service/
// sweep_r3s2_numa_pinned.jsonl).  The thread's memory policy is set to
// prefer that node around the allocation and its first touch, then restored.
hipError_t host_alloc_on_node(void **p, size_t bytes, unsigned flags, int node) {
    constexpr int kMpolPreferred = 1;
    constexpr unsigned long kMaxNode = 1024;
    unsigned long old_mask[kMaxNode / (8 * sizeof(unsigned long))] = {0};
    int old_mode = 0;
    bool moved = false;
    if (node >= 0 && node < static_cast<int>(kMaxNode) &&
        syscall(SYS_get_mempolicy, &old_mode, old_mask, kMaxNode, nullptr, 0ul) == 0) {
        unsigned long mask[kMaxNode / (8 * sizeof(unsigned long))] = {0};
        mask[node / (8 * sizeof(unsigned long))] = 1ul << (node % (8 * sizeof(unsigned long)));
        moved = syscall(SYS_set_mempolicy, kMpolPreferred, mask, kMaxNode) == 0;
    }
    hipError_t e = hipHostMalloc(p, bytes, flags | (moved ? hipHostMallocNumaUser : 0u));
    if (e == hipSuccess) std::memset(*p, 0, bytes);  // first touch under the policy
    if (moved) (void)syscall(SYS_set_mempolicy, old_mode, old_mode ? old_mask : nullptr, old_mode ? kMaxNode : 0ul);
    return e;
}

}  // namespace

extern "C" {

// nffacl_local_device: group.cpp (it spreads a node's callers over the node's devices)

int nffacl_device_numa_node(int hip_device) {
    const DeviceNodes &dn = device_nodes();
    if (dn.count <= 0) return NFFACL_ERR_NO_DEVICE;
    if (hip_device < 0 || hip_device >= dn.count) return NFFACL_ERR_INVALID_ARG;
    return dn.node[hip_device] >= 0 ? dn.node[hip_device] : NFFACL_ERR_HIP;
}

int nffacl_rules_prepare(const nffacl_rules *rules, int hip_device) {
    int st = NFFACL_OK;
    (void)rules_table(rules, hip_device, st);
    return st;
}

}  // extern "C"

namespace {

int service_create(int hip_device, uint32_t mailboxes, uint32_t idle_us, bool burst, nffacl_service **out) {
    if (!out) return NFFACL_ERR_INVALID_ARG;
    *out = nullptr;
    if (mailboxes == 0) {  // default: 128 scalar / 64 burst mailboxes (NFFACL_TUNE_SVC_MAILBOXES)
        long v = 0;
        bool set = false;
        std::string err;
        if (!env_knob("NFFACL_TUNE_SVC_MAILBOXES", burst ? 1 : 64, 4096, v, set, err)) {
            set_last_error(err);
            return NFFACL_ERR_INVALID_ARG;
        }
        mailboxes = set ? static_cast<uint32_t>(v) : burst ? 64u : 128u;
    }
    if ((!burst && mailboxes % 64 != 0) || mailboxes > (burst ? 1024u : 4096u) || idle_us > 10000000u)
        return NFFACL_ERR_INVALID_ARG;
    if (idle_us == 0) idle_us = 2000;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        (void)hipGetLastError();
        set_last_error("no HIP device visible");
        return NFFACL_ERR_NO_DEVICE;
    }
    if (hip_device < 0 || hip_device >= count || hip_device >= kMaxDevices) return NFFACL_ERR_INVALID_ARG;
    HIP_TRY(hipSetDevice(hip_device));
    int khz = 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, hip_device) != hipSuccess || khz <= 0) {
        (void)hipGetLastError();
        khz = 100000;  // gfx9 s_memrealtime: 100 MHz
    }
    nffacl_service *s = new (std::nothrow) nffacl_service();
    if (!s) return NFFACL_ERR_NOMEM;
    s->device = hip_device;
    s->id = g_next_id.fetch_add(1, std::memory_order_relaxed);
    s->n_mb = mailboxes;
    s->burst = burst;
    s->box_stride = burst ? kSvcBurstBoxBytes : kSvcBoxBytes;
    s->resp_stride = burst ? kSvcBurstRespWords : kSvcRespStride;
    s->mbx.reset(new (std::nothrow) MailboxState[mailboxes]);
    const size_t box_bytes = size_t(mailboxes) * s->box_stride;
    const size_t bell_bytes = (size_t(mailboxes) * 4 + 255) / 256 * 256;
    const size_t resp_bytes = size_t(mailboxes) * s->resp_stride * 8;
    const size_t stat_bytes = size_t(s->waves()) * kSvcStatWords * 8;
    const size_t bytes = box_bytes + bell_bytes + resp_bytes + 64 + stat_bytes;
    hipError_t e = s->mbx ? hipSuccess : hipErrorOutOfMemory;
    // NFFACL_TUNE_SVC_NODE=0: the caller's default memory policy instead of the device's node
    const char *node_env = std::getenv("NFFACL_TUNE_SVC_NODE");
    const bool on_node = !(node_env && node_env[0] == '0' && node_env[1] == 0);
    if (e == hipSuccess)
        e = host_alloc_on_node(reinterpret_cast<void **>(&s->h_mem), bytes, hipHostMallocMapped | hipHostMallocCoherent,
                               on_node && hip_device < device_nodes().count ? device_nodes().node[hip_device] : -1);
    uint8_t *d_mem = nullptr;
    if (e == hipSuccess) e = hipHostGetDevicePointer(reinterpret_cast<void **>(&d_mem), s->h_mem, 0);
    // NFFACL_TUNE_SVC_HOSTPTR=1 (experiment): the kernels use the host pointer itself (unified addressing)
    const char *hp_env = std::getenv("NFFACL_TUNE_SVC_HOSTPTR");
    if (e == hipSuccess && hp_env && hp_env[0] == '1') d_mem = s->h_mem;
    int lo = 0, hi = 0;
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&lo, &hi);
    // its own (highest-priority) stream: kept off the queues of batch work
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, hi);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s->done, hipEventDisableTiming);
    if (e != hipSuccess) {
        set_last_error(std::string("service: ") + hipGetErrorString(e));
        release_service(s);
        return e == hipErrorOutOfMemory ? NFFACL_ERR_NOMEM : NFFACL_ERR_HIP;
    }
    std::memset(s->h_mem, 0, bytes);
    s->h_box = s->h_mem;
    s->h_bell = reinterpret_cast<uint32_t *>(s->h_mem + box_bytes);
    const size_t rb = box_bytes + bell_bytes;  // responses from here
    s->h_resp = reinterpret_cast<uint64_t *>(s->h_mem + rb);
    s->h_ctrl = reinterpret_cast<uint32_t *>(s->h_mem + rb + resp_bytes);
    const uint64_t tpu = uint64_t(khz) / 1000;  // ticks per µs
    s->ticks_per_us = tpu;
    s->args.box = d_mem;
    s->args.resp = reinterpret_cast<uint64_t *>(d_mem + rb);
    s->args.ctrl = reinterpret_cast<uint32_t *>(d_mem + rb + resp_bytes);
    s->args.stats = reinterpret_cast<uint64_t *>(d_mem + rb + resp_bytes + 64);
    s->h_stats = reinterpret_cast<uint64_t *>(s->h_mem + rb + resp_bytes + 64);
    s->args.box_bytes = static_cast<uint32_t>(box_bytes);
    s->args.range_bytes = static_cast<uint32_t>(rb);
    s->args.idle_ticks = uint64_t(idle_us) * tpu;
    s->args.hot_ticks = 200 * tpu;
    s->args.life_ticks = 100000 * tpu;  // 100 ms, then the armer re-launches if calls keep coming
    // INDEXED tables up to 64 KiB (C1/C2-class) are staged in the consumer's
    // LDS (NFFACL_TUNE_SVC_LDS=0: walk every table from global memory)
    s->args.lds_dwords = kSvcLdsDwords;
    {
        long v = 0;
        bool set = false;
        std::string err;
        if (!env_knob("NFFACL_TUNE_SVC_LDS", 0, 1, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        if (set && v == 0) s->args.lds_dwords = 0;
        // Callers sleep through most of the PCIe round trip instead of
        // spinning it: under a CPU quota a spinning caller burns the quota the
        // other callers need (throughput = quota / CPU time per call)
        if (!env_knob("NFFACL_TUNE_SVC_SLEEP_NS", -1, 100000, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        if (set) s->sleep_ns = static_cast<int32_t>(v);
        if (!env_knob("NFFACL_TUNE_SVC_TIMEOUT_US", 1000, 10000000, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        if (set) s->timeout_us = static_cast<uint64_t>(v);
        if (!env_knob("NFFACL_TUNE_SVC_NT", 0, 1, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        if (set) s->nt = v != 0;
        if (!env_knob("NFFACL_TUNE_SVC_FULLPOLL", 0, 1, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        s->args.full_poll = !set || v != 0 ? 1u : 0u;
        if (!env_knob("NFFACL_TUNE_SVC_IDLE_NAPS", 0, 1000, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        s->args.idle_naps = set ? static_cast<uint32_t>(v) : 0u;
        if (!env_knob("NFFACL_TUNE_SVC_POST_NAPS", 0, 200, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        s->args.post_naps = set ? static_cast<uint32_t>(v) : 12u;
        if (!env_knob("NFFACL_TUNE_SVC_NAP_ADAPT", 0, 1, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        s->args.nap_adapt = !set || v != 0 ? 1u : 0u;
        if (!env_knob("NFFACL_TUNE_SVC_TRACE", 0, 1, v, set, err)) {
            set_last_error(err);
            release_service(s);
            return NFFACL_ERR_INVALID_ARG;
        }
        s->trace = set && v != 0;
        s->cpus = cpu_budget();
    }
    const void *kern = burst ? reinterpret_cast<const void *>(dev::k_service_burst)
                             : reinterpret_cast<const void *>(dev::k_service);
    if (s->args.lds_dwords &&
        hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(s->args.lds_dwords * 4)) !=
            hipSuccess) {
        (void)hipGetLastError();
        s->args.lds_dwords = 0;
    }
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        if (!g_live) {
            g_live = new std::set<nffacl_service *>();
            std::atexit(stop_all_at_exit);
        }
        g_live->insert(s);
    }
    s->armer = std::thread(armer_main, s);
    *out = s;
    return NFFACL_OK;
}

// One request through mailbox `mb` (its lock held by the caller): `post(tag,
// key)` writes the request's chunks with `tag` and the table key (the
// descriptor's generation, or kSvcWithdrawn), `answered(tag)` tells whether
// every response word of the request carries `tag`.
//
// Failure policy (the reference's verdict path never errors, acl.go:522-565):
// a caller that has no answer after timeout_us re-posts its request under a
// new tag and re-arms the consumer (counted in `retries`); if that one is not
// answered within timeout_us either, it WITHDRAWS the request — rewrites it
// with the key kSvcWithdrawn, which the consumer answers without reading any
// table — records the table's use on the consumer's stream (the table's
// retirement then waits for the consumer launch that may still hold the old
// request) and returns NFFACL_ERR_TIMEOUT (counted in `timeouts`); the
// caller's verdict is then 0 (reject), the value l3ACL gives a packet no rule
// matches.  Later calls are served normally once the consumer runs again.
template <class Post, class Answered>
int post_and_wait(nffacl_service *s, MailboxState &m, uint32_t mb, DevTable *t, uint32_t key, Post post,
                  Answered answered) {
    for (int attempt = 0;; ++attempt) {
        const uint32_t tag = ++m.seq;
        const Clock::time_point tp0 = s->trace ? Clock::now() : Clock::time_point{};
        post(tag, key);
        if (s->nt) _mm_sfence();  // the streaming stores are visible before the bell
        __atomic_store_n(&s->h_bell[mb], tag, __ATOMIC_RELEASE);  // idle waves watch the bells
        std::atomic_thread_fence(std::memory_order_seq_cst);      // request visible before `running` is read
        if (!s->running.load(std::memory_order_seq_cst)) kick(s);
        const Clock::time_point tp1 = s->trace ? Clock::now() : Clock::time_point{};
        // sleep first?  (adaptive: only with more callers than CPUs)
        const bool adaptive = s->sleep_ns < 0 && s->next_mb.load(std::memory_order_relaxed) > s->cpus;
        const uint32_t nap = attempt ? 0u : adaptive ? m.nap : s->sleep_ns > 0 ? static_cast<uint32_t>(s->sleep_ns) : 0u;
        Clock::time_point woke{};
        if (nap) {
            thread_local bool slack = false;
            if (!slack) {  // hrtimer wake-ups at the requested time (default slack: 50 us)
                (void)prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);
                slack = true;
            }
            const timespec ts{0, static_cast<long>(nap)};
            (void)nanosleep(&ts, nullptr);
        }
        if (adaptive) woke = Clock::now();
        bool spun = false;
        uint32_t spins = 0;
        Clock::time_point t0{};
        int st = NFFACL_OK;
        while (true) {
            if (answered(tag)) break;
            spun = true;
            _mm_pause();
            if ((++spins & 1023u) == 0) {
                const Clock::time_point now = Clock::now();
                if (spins == 1024) t0 = now;
                if ((st = s->error.load(std::memory_order_acquire)) != NFFACL_OK) break;
                if (!s->running.load(std::memory_order_seq_cst)) kick(s);
                if (now - t0 > std::chrono::microseconds(s->timeout_us)) {
                    st = NFFACL_ERR_TIMEOUT;
                    break;
                }
            }
        }
        if (st == NFFACL_OK && s->trace) {
            const Clock::time_point tp2 = Clock::now();
            s->tr_post_ns.fetch_add(uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(tp1 - tp0).count()),
                                    std::memory_order_relaxed);
            s->tr_wait_ns.fetch_add(uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(tp2 - tp1).count()),
                                    std::memory_order_relaxed);
            s->tr_spins.fetch_add(spins, std::memory_order_relaxed);
        }
        if (st == NFFACL_OK) {
            if (adaptive && attempt == 0) {
                // Aim the nap short of the answer (an oversleep costs the whole
                // wake-up time, a short spin only CPU): an answer already there
                // at wake-up cuts it by a quarter; a spin after waking lengthens
                // it by a quarter of the spin beyond 300 ns, at most 500 ns per
                // call (a caller preempted while spinning must not drag it up).
                if (!spun) {
                    m.nap -= std::max(m.nap / 4u, std::min(m.nap, 100u));
                } else {
                    const int64_t spin =
                        std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - woke).count();
                    if (spin > 300)
                        m.nap = std::min(m.nap + static_cast<uint32_t>(std::min<int64_t>((spin - 300) / 4, 500)), 20000u);
                }
            }
            return NFFACL_OK;
        }
        if (st != NFFACL_ERR_TIMEOUT) return st;  // the consumer failed (sticky HIP error)
        if (attempt == 0) {
            s->retries.fetch_add(1, std::memory_order_relaxed);
            continue;  // re-post under a new tag, re-arm
        }
        // withdraw: same tag, no table; the table's retirement waits for the
        // consumer launch that may still hold the request
        post(tag, kSvcWithdrawn);
        if (s->nt) _mm_sfence();
        std::atomic_thread_fence(std::memory_order_seq_cst);
        (void)t->note_use(s->stream);
        s->timeouts.fetch_add(1, std::memory_order_relaxed);
        set_last_error("service: no answer within the timeout (twice); request withdrawn, verdict 0");
        return NFFACL_ERR_TIMEOUT;
    }
}

inline void put16(__m128i *dst, __m128i v, bool nt) {
    if (nt) _mm_stream_si128(dst, v);
    else _mm_store_si128(dst, v);
}

// One packet as chunk payload (service.hpp): bytes [0, min(len, 80)), zero
// after, 12 per chunk with the tag in word 3.  A whole 80-byte prefix is read
// straight from the frame (chunks 0-5: 16-byte loads ending at byte 76; chunk
// 6: bytes 72-79); shorter frames go through a zeroed copy.  (Round 4: the
// byte-wise copy took 2.4 us per 32-packet burst on the host — a third of a
// burst call — against 0.2-0.5 us for this.)
inline void packet_chunks(const uint8_t *frame, uint32_t len, uint32_t tag, __m128i *dst, bool nt) {
    static_assert(kSvcPktChunks == 7 && kSvcSlot == 80, "six 16-byte loads + one 8-byte load per packet");
    const __m128i keep = _mm_set_epi32(0, -1, -1, -1);
    const __m128i t = _mm_set_epi32(static_cast<int>(tag), 0, 0, 0);
    alignas(16) uint8_t b[96];
    const uint8_t *src = frame;
    if (len < kSvcSlot) {
        std::memset(b, 0, sizeof b);
        if (len) std::memcpy(b, frame, len);
        src = b;
    }
    for (uint32_t j = 0; j + 1 < kSvcPktChunks; ++j) {
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 12 * j));
        put16(dst + j, _mm_or_si128(_mm_and_si128(v, keep), t), nt);
    }
    // bytes 72-79, then zeros (80-83) and the tag
    const __m128i last = _mm_loadl_epi64(reinterpret_cast<const __m128i *>(src + 12 * (kSvcPktChunks - 1)));
    put16(dst + kSvcPktChunks - 1, _mm_or_si128(last, t), nt);
}

// One packet as burst-mailbox payload (service.hpp): bytes [12, min(len, 80)),
// zero after, 12 per chunk with the tag in word 3 — packet_chunks without its
// first chunk (the MAC addresses).
inline void burst_chunks(const uint8_t *frame, uint32_t len, uint32_t tag, __m128i *dst, bool nt) {
    static_assert(kSvcBurstPktChunks == 6 && kSvcSlot == 80, "five 16-byte loads + one 8-byte load per packet");
    const __m128i keep = _mm_set_epi32(0, -1, -1, -1);
    const __m128i t = _mm_set_epi32(static_cast<int>(tag), 0, 0, 0);
    alignas(16) uint8_t b[96];
    const uint8_t *src = frame;
    if (len < kSvcSlot) {
        std::memset(b, 0, sizeof b);
        if (len) std::memcpy(b, frame, len);
        src = b;
    }
    for (uint32_t j = 0; j + 1 < kSvcBurstPktChunks; ++j) {  // bytes 12 + 12j .. +15
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 12 + 12 * j));
        put16(dst + j, _mm_or_si128(_mm_and_si128(v, keep), t), nt);
    }
    // bytes 72-79, then zeros (80-83) and the tag
    const __m128i last = _mm_loadl_epi64(reinterpret_cast<const __m128i *>(src + 72));
    put16(dst + kSvcBurstPktChunks - 1, _mm_or_si128(last, t), nt);
}

inline void store_chunk(__m128i *dst, uint32_t x, uint32_t y, uint32_t z, uint32_t w, bool nt) {
    put16(dst, _mm_set_epi32(static_cast<int>(w), static_cast<int>(z), static_cast<int>(y), static_cast<int>(x)), nt);
}

}  // namespace

extern "C" {

int nffacl_service_create(int hip_device, uint32_t mailboxes, uint32_t idle_us, nffacl_service **out) {
    return service_create(hip_device, mailboxes, idle_us, false, out);
}

int nffacl_service_create_burst(int hip_device, uint32_t mailboxes, uint32_t idle_us, nffacl_service **out) {
    return service_create(hip_device, mailboxes, idle_us, true, out);
}

int nffacl_service_classify(nffacl_service *s, const nffacl_rules *rules, const uint8_t *frame, uint32_t len,
                            uint32_t flags, uint32_t *port) {
    if (!s || !rules || (!frame && len) || (flags & ~uint32_t(NFFACL_PARSE_VLAN)) != 0) return NFFACL_ERR_INVALID_ARG;
    if (s->burst) return nffacl_service_classify_burst(s, rules, &frame, &len, 1, flags, port);
    auto failed = [s](int st) {
        std::lock_guard<std::mutex> g(s->mu);
        set_last_error(s->error_msg);
        return st;
    };
    int st = s->error.load(std::memory_order_acquire);
    if (st != NFFACL_OK) return failed(st);
    DevTable *t = rules_table(rules, s->device, st);
    if (!t) return st;
    if (t->svc_kind == kSvcNone) return NFFACL_ERR_UNSUPPORTED;
    const uint32_t mb = my_mailbox(s);
    MailboxState &m = s->mbx[mb];
    while (m.lock.exchange(1, std::memory_order_acquire) != 0) _mm_pause();
    __m128i *dst = reinterpret_cast<__m128i *>(s->h_box + size_t(mb) * kSvcBoxBytes);
    const uint64_t desc = reinterpret_cast<uint64_t>(t->d_desc);
    const uint32_t live_key = t->gen << 1 | (flags & NFFACL_PARSE_VLAN ? 1u : 0u);
    const uint64_t *r = s->h_resp + size_t(mb) * kSvcRespStride;
    uint64_t v = 0;
    st = post_and_wait(
        s, m, mb, t, live_key,
        [&](uint32_t tag, uint32_t key) {
            // the eight chunks (service.hpp), ascending: the tag chunk last (x86 stores stay in order)
            packet_chunks(frame, len, tag, dst, s->nt);
            if (key == kSvcWithdrawn) store_chunk(dst + kSvcPktChunks, 0, 0, key, tag, s->nt);
            else store_chunk(dst + kSvcPktChunks, static_cast<uint32_t>(desc), static_cast<uint32_t>(desc >> 32), key, tag,
                             s->nt);
        },
        [&](uint32_t tag) {
            v = __atomic_load_n(r, __ATOMIC_ACQUIRE);
            return static_cast<uint32_t>(v >> 32) == tag;
        });
    m.lock.store(0, std::memory_order_release);
    if (st == NFFACL_ERR_HIP) return failed(st);
    if (st == NFFACL_ERR_TIMEOUT) {
        if (port) *port = 0;
        return st;
    }
    if (st != NFFACL_OK) return st;
    s->requests.fetch_add(1, std::memory_order_relaxed);
    if (port) *port = static_cast<uint32_t>(v);
    return NFFACL_OK;
}

int nffacl_service_classify_burst(nffacl_service *s, const nffacl_rules *rules, const uint8_t *const *frames,
                                  const uint32_t *lens, uint32_t n, uint32_t flags, uint32_t *ports) {
    if (!s || !rules || !s->burst || n > kSvcBurstMax || (n && (!frames || !ports)) ||
        (flags & ~uint32_t(NFFACL_PARSE_VLAN)) != 0)
        return NFFACL_ERR_INVALID_ARG;
    if (n == 0) return NFFACL_OK;
    const Clock::time_point tc0 = s->trace ? Clock::now() : Clock::time_point{};
    for (uint32_t i = 0; i < n; ++i)
        if (!frames[i] && (!lens || lens[i])) return NFFACL_ERR_INVALID_ARG;
    auto failed = [s](int st) {
        std::lock_guard<std::mutex> g(s->mu);
        set_last_error(s->error_msg);
        return st;
    };
    int st = s->error.load(std::memory_order_acquire);
    if (st != NFFACL_OK) return failed(st);
    DevTable *t = rules_table(rules, s->device, st);
    if (!t) return st;
    if (t->svc_kind == kSvcNone) return NFFACL_ERR_UNSUPPORTED;
    const uint32_t mb = my_mailbox(s);
    MailboxState &m = s->mbx[mb];
    while (m.lock.exchange(1, std::memory_order_acquire) != 0) _mm_pause();
    __m128i *dst = reinterpret_cast<__m128i *>(s->h_box + size_t(mb) * kSvcBurstBoxBytes);
    const uint64_t desc = reinterpret_cast<uint64_t>(t->d_desc);
    const uint32_t live_key = t->gen << 1 | (flags & NFFACL_PARSE_VLAN ? 1u : 0u);
    const uint64_t *r = s->h_resp + size_t(mb) * kSvcBurstRespWords;
    st = post_and_wait(
        s, m, mb, t, live_key,
        [&](uint32_t tag, uint32_t key) {
            const bool wd = key == kSvcWithdrawn;
            const uint32_t cnt = wd ? 1u : n;
            for (uint32_t i = 0; i < cnt; ++i)
                burst_chunks(wd ? nullptr : frames[i], wd ? 0u : lens ? lens[i] : kSvcSlot, tag,
                             dst + kSvcBurstHdrChunks + kSvcBurstPktChunks * i, s->nt);
            store_chunk(dst + 1, cnt, 0, 0, tag, s->nt);
            // the consumer reads the packets only once the header carries the
            // tag: the header chunk goes last (streaming stores: after a fence)
            if (s->nt) _mm_sfence();
            if (wd) store_chunk(dst, 0, 0, key, tag, s->nt);
            else store_chunk(dst, static_cast<uint32_t>(desc), static_cast<uint32_t>(desc >> 32), key, tag, s->nt);
        },
        [&](uint32_t tag) {
            // spin on one word, then check all (the words arrive in any order)
            // (round 4: 16 clones 68.9 vs 66.4 Mpps checking all 32 words every spin,
            // profiles/r4_service/trace/spin1_*)
            if (static_cast<uint32_t>(__atomic_load_n(r + n - 1, __ATOMIC_ACQUIRE) >> 32) != tag) return false;
            for (uint32_t i = n; i-- > 0;)
                if (static_cast<uint32_t>(__atomic_load_n(r + i, __ATOMIC_ACQUIRE) >> 32) != tag) return false;
            return true;
        });
    m.lock.store(0, std::memory_order_release);
    if (st == NFFACL_ERR_HIP) return failed(st);
    if (st == NFFACL_ERR_TIMEOUT) {
        std::memset(ports, 0, size_t(n) * 4);
        return st;
    }
    if (st != NFFACL_OK) return st;
    for (uint32_t i = 0; i < n; ++i) ports[i] = static_cast<uint32_t>(__atomic_load_n(r + i, __ATOMIC_RELAXED));
    s->requests.fetch_add(n, std::memory_order_relaxed);
    if (s->trace) {
        s->tr_calls.fetch_add(1, std::memory_order_relaxed);
        s->tr_total_ns.fetch_add(
            uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - tc0).count()),
            std::memory_order_relaxed);
    }
    return NFFACL_OK;
}

int nffacl_service_pause(nffacl_service *s, int paused) {
    if (!s) return NFFACL_ERR_INVALID_ARG;
    if (paused) {
        s->paused.store(true, std::memory_order_release);
        __atomic_store_n(s->h_ctrl, 1u, __ATOMIC_RELEASE);  // the resident consumer leaves
        return NFFACL_OK;
    }
    {
        std::lock_guard<std::mutex> g(s->mu);
        if (s->stop) return NFFACL_ERR_INVALID_ARG;
    }
    // The consumer of the pause has left once `running` drops (still paused,
    // the armer launches none meanwhile); then clear the stop word, unpause
    // and re-arm.  A resume that gives up leaves the service consistently
    // paused (stop word set, `paused` true) for a later resume to finish.
    const auto limit = Clock::now() + std::chrono::seconds(2);
    while (s->running.load(std::memory_order_seq_cst) && Clock::now() < limit) std::this_thread::yield();
    if (s->running.load(std::memory_order_seq_cst)) return NFFACL_ERR_TIMEOUT;
    __atomic_store_n(s->h_ctrl, 0u, __ATOMIC_RELEASE);
    {
        std::lock_guard<std::mutex> g(s->mu);
        if (s->stop) return NFFACL_ERR_INVALID_ARG;
        s->paused.store(false, std::memory_order_release);
    }
    kick(s);
    return NFFACL_OK;
}

int nffacl_service_get_stats(nffacl_service *s, nffacl_service_stats *out) {
    if (!s || !out) return NFFACL_ERR_INVALID_ARG;
    out->launches = s->launches.load(std::memory_order_relaxed);
    out->retries = s->retries.load(std::memory_order_relaxed);
    out->requests = s->requests.load(std::memory_order_relaxed);
    out->timeouts = s->timeouts.load(std::memory_order_relaxed);
    out->running = s->running.load(std::memory_order_relaxed) ? 1u : 0u;
    out->table_oob = __atomic_load_n(&s->h_ctrl[2], __ATOMIC_ACQUIRE);
    std::lock_guard<std::mutex> g(s->mu);
    const double tpu = double(s->ticks_per_us);
    out->polls = s->acc[0];
    out->poll_ns = s->acc[0] ? s->acc[1] * 1000.0 / tpu / double(s->acc[0]) : 0.0;
    out->groups = s->acc[2];
    out->group_ns = s->acc[2] ? s->acc[3] * 1000.0 / tpu / double(s->acc[2]) : 0.0;
    out->answered = s->acc[4];
    out->torn = s->acc[5];
    return NFFACL_OK;
}

void nffacl_service_destroy(nffacl_service *s) {
    if (!s) return;
    {
        std::lock_guard<std::mutex> g(g_live_mu);
        if (g_live) g_live->erase(s);
    }
    stop_kernel(s);
    (void)hipSetDevice(s->device);
    (void)hipStreamSynchronize(s->stream);
    release_service(s);
}

}  // extern "C"
