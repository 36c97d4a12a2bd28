// engine.hip — HIP kernels (gfx950 / CDNA4) and the device engine of libnffacl.
//
// Hot path replaced: (*Packet).l3ACL, packet/acl.go:522-565 (+ l4ACL :508-520,
// ParseAllKnownL3 packet/packet.go:353-363, ParseL4ForIPv4/6 :278-285), run
// over a batch of packets resident in HBM instead of one mbuf at a time.
//
// Execution model (one wave64 = 64 consecutive packets, one packet per lane):
//  * each lane loads its 64-byte slot with four 16-byte loads and extracts the
//    header fields with funnel shifts (every field after the Ethernet header
//    is at a wire offset = 2 mod 4);
//  * LINEAR: the rule records are wave-uniform, so they stream through the
//    scalar data cache (s_load) and every rule costs a handful of VALU ops
//    on all 64 packets at once; a 64-bit ballot of still-undecided lanes ends
//    the scan as soon as every packet of the wave has its first match;
//  * INDEXED: see classify_indexed() — per-lane interval search + ordered
//    candidate lists, tables staged in LDS;
//  * the verdict vector is written as one u32 port per packet (coalesced) and
//    one 64-bit permit word per wave (ballot of port > 0).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include "classify.hpp"
#include "compile.hpp"
#include "devutil.hpp"
#include "engine.hpp"
#include "service.hpp"

namespace nffacl {

thread_local std::string g_last_error;

void set_last_error(const std::string &s) { g_last_error = s; }
const char *last_error() { return g_last_error.c_str(); }

namespace dev {

__global__ void __launch_bounds__(256)
k_linear_slots(const uint8_t *__restrict__ slots, uint32_t stride, uint64_t n, LinearArgs a,
               uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    NFFACL_WAVE_LOOP(n) {
        const uint64_t idx = base + lane;
        const bool live = idx < n;
        const uint8_t *pkt = slots + (live ? idx : 0) * stride;
        uint32_t d[16];
        load16(pkt, d);
        Fields f;
        parse_fields(d, live, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
            far_dwords(pkt, stride, k, lo, hi);
        }, a.flags);
        const uint32_t res = classify_linear(f, a.rec4, a.n4, a.rec6, a.n6);
        store_verdicts(base, lane, live, res, port_out, permit_out);
    }
}

// Packed frames: desc = offset << 16 | length; bytes >= length read as 0.
__global__ void __launch_bounds__(256)
k_linear_frames(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint64_t n,
                LinearArgs a, uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    NFFACL_WAVE_LOOP(n) {
        const uint64_t idx = base + lane;
        const bool live = idx < n;
        const uint64_t ds = live ? desc[idx] : 0;
        const uint32_t len = static_cast<uint32_t>(ds & 0xFFFFu);
        const uint8_t *pkt = frames + (ds >> 16);
        uint32_t d[16];
        load16_frame(pkt, len, d);
        Fields f;
        parse_fields(d, live, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
            far_dwords(pkt, len, k, lo, hi);
        }, a.flags);
        const uint32_t res = classify_linear(f, a.rec4, a.n4, a.rec6, a.n6);
        store_verdicts(base, lane, live, res, port_out, permit_out);
    }
}


// `pf`: the next batch's packet loads (load mode 6); the pipelined walk
// issues them itself, after its first window's tests; other walks up front.
template <int NS, int TM, class PF>
__device__ __forceinline__ uint32_t classify_any(const IndexedArgs &a, const Fields &f, PF &&pf) {
    if constexpr (TM == kTabFlatLdsP) {
        FlatScratch<4> *W = reinterpret_cast<FlatScratch<4> *>(lds_tab + a.stage_dwords);
        return classify_flat_pipe<NS>(a, f, W[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)], lane_id(), pf);
    }
    pf();
    if (TM == kTabFlat || TM == kTabFlat4) {
        constexpr int R = TM == kTabFlat4 ? 4 : 2;
        FlatScratch<R> *W = reinterpret_cast<FlatScratch<R> *>(lds_tab);
        const uint32_t lane = lane_id();
        return classify_flat<NS, R, false>(a, f, W[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)], lane);
    }
    if (TM == kTabFlatLds || TM == kTabFlatLds4 || TM == kTabFlatLds4U || TM == kTabFlatLdsG) {
        // scratch after the staged directories (stage_dwords: multiple of 4)
        constexpr int R = TM == kTabFlatLds ? 2 : 4;
        FlatScratch<R> *W = reinterpret_cast<FlatScratch<R> *>(lds_tab + a.stage_dwords);
        const uint32_t lane = lane_id();
        return classify_flat<NS, R, true, TM == kTabFlatLds4U || TM == kTabFlatLdsG, true, TM == kTabFlatLdsG>(
            a, f, W[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)], lane);
    }
    if constexpr (NS <= 4) {  // per-lane walks: the positional four slots
        if (TM == kTabLds) return classify_indexed<NS, 1>(LdsTab{}, a, f);
        if (TM == kTabLdsNP) return classify_indexed<NS, 1, LdsTab, true>(LdsTab{}, a, f);
        if (TM == kTabSplit) return classify_indexed<NS, 1>(SplitTab{a.tab}, a, f);
        return classify_indexed<NS, 1>(GlobalTab{a.tab}, a, f);
    }
    return 0u;
}

// Which 64-packet batches a wave classifies.  heads == nullptr: a fixed grid
// stride from the wave's global index.  Otherwise batches are pulled at run
// time, so that a workgroup that starts late (its CU held by a resident
// consumer, service.hip) takes fewer of them instead of stretching the
// launch by a whole share.  Eight pull heads, one per group of workgroups
// sharing an XCD (blockIdx % 8: a label, never relied on for correctness),
// each own 1/8 of the batches.  A head's range opens with one static chunk
// per wave of its group, of 1 + (j % 8) batches for the group's j-th wave
// (no pull at the start, and the staggered lengths spread the group's first
// pulls over time: a head takes ~88 pulls per microsecond,
// MI355X_MICROARCH.md "dequeue"; short, so that a late wave's chunk is a
// short tail); then one returning atomicAdd on the head
// takes up to dyn_g batches (a guided size, smaller as the head drains,
// never below dyn_gmin), and a wave whose head is drained pulls from the
// other seven.  The last wave to finish zeroes the heads for the next
// launch on the same stream (dyn_heads: one block per stream).
// (Round 5: the pull's result read a chunk later, its latency hidden, made
// the compiler carry the batch state per lane and classify wrong batches;
// the pull is read at once.)
struct BatchSource {
    uint32_t *heads;
    uint64_t nb, b, end, step;  // batches; the current chunk [b, end); the grid stride
    uint32_t home, tried, g, gmax, gmin, wpx, wpb, groups;

    // waves of group x, and the batches their static chunks take
    __device__ uint64_t group_waves(uint32_t x) const { return x < groups ? uint64_t((groups - 1 - x) / 8 + 1) * wpb : 0; }
    __device__ static uint64_t static_len(uint64_t j) {  // sum over waves i < j of (1 + i % 8)
        const uint64_t r = j & 7u;
        return j + (j >> 3) * 28u + r * (r - 1) / 2;
    }
    __device__ uint32_t pull(uint32_t x, uint32_t n) const {
        uint32_t s = 0;
        if (lane_id() == 0) s = atomicAdd(heads + x * kDynHeadStride, n);
        return __builtin_amdgcn_readfirstlane(s);
    }
    // the next chunk from the heads (b = end = nb when all are drained)
    __device__ void refill() {
        while (tried < 8) {
            const uint32_t x = (home + tried) & 7u;
            const uint64_t lo = (nb * x >> 3) + static_len(group_waves(x)), hi = nb * (x + 1) >> 3;
            if (lo < hi) {
                const uint64_t s = lo + pull(x, g);
                if (s < hi) {
                    b = s;
                    end = s + g < hi ? s + g : hi;
                    const uint64_t per = (hi - end) / (2u * wpx);
                    g = per < gmin ? gmin : per > gmax ? gmax : static_cast<uint32_t>(per);
                    return;
                }
            }
            ++tried;
        }
        b = end = nb;
    }
    // packet index of the wave's first batch (>= n: none)
    __device__ uint64_t first(uint32_t *h, uint64_t n, const IndexedArgs &a, uint64_t wave, uint64_t waves) {
        heads = h;
        nb = (n + 63) >> 6;
        if (!heads) {
            b = wave;
            step = waves;
            return b * 64;
        }
        home = blockIdx.x & 7u;
        tried = 0;
        gmax = g = a.dyn_g;
        gmin = a.dyn_gmin;
        wpx = a.dyn_wpx;
        wpb = blockDim.x >> 6;
        groups = gridDim.x;
        // this wave's static chunk: the j-th of its group
        const uint64_t j = uint64_t(blockIdx.x >> 3) * wpb + (wave - uint64_t(blockIdx.x) * wpb);
        const uint64_t hi = nb * (home + 1) >> 3;
        b = (nb * home >> 3) + static_len(j);
        end = b + 1 + (j & 7u);
        if (end > hi) end = hi;
        if (b >= end) refill();
        return b * 64;
    }
    __device__ uint64_t next() {
        if (!heads) {
            b += step;
        } else if (++b >= end) {
            refill();
        }
        return b * 64;
    }
    // every wave, after its last batch: the last one resets the heads
    __device__ void finish(uint64_t waves) const {
        if (!heads) return;
        uint32_t c = 0;
        if (lane_id() == 0) c = atomicAdd(heads + 8 * kDynHeadStride, 1u);
        c = __builtin_amdgcn_readfirstlane(c);
        if (c == waves - 1 && lane_id() <= 8)
            __hip_atomic_store(heads + lane_id() * kDynHeadStride, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
};

// Batches of 64 packets (BatchSource: a grid stride or, load mode 4, pulled).
//  * rows (any stride): the next batch's 64-byte rows are loaded while the
//    current batch is classified (software pipelining, 16 VGPRs);
//  * COAL (stride == 64): lane-contiguous loads + quad transpose, lane l
//    classifying packet coal_packet(l) of its wave's batch; no register
//    prefetch (it would push the kernel past 64 VGPRs, i.e. below 8 waves per
//    SIMD) — 32 resident waves per CU keep 128 KiB of loads in flight.
// (experiment builds: NFFACL_EXP_MAXVGPR / _MAXSGPR cap the slot kernels'
// registers.  Round 6: C2's kernel holds 87 SGPRs, past the 80 that admit 8
// waves per SIMD (MI355X_MICROARCH.md, residency); capped at 80 (78, 7 SGPR
// spills) it ran 0.2109 / 0.2091 vs 0.2061 / 0.2063 ms, profiles/r6_ab/s80/)
#ifdef NFFACL_EXP_MAXVGPR
#define NFFACL_SLOTS_VGPR __attribute__((amdgpu_num_vgpr(NFFACL_EXP_MAXVGPR)))
#elif defined(NFFACL_EXP_MAXSGPR)
#define NFFACL_SLOTS_VGPR __attribute__((amdgpu_num_sgpr(NFFACL_EXP_MAXSGPR)))
#else
#define NFFACL_SLOTS_VGPR
#endif
template <int NS, int TM, int MODE>
__global__ void __launch_bounds__(1024) NFFACL_SLOTS_VGPR
k_indexed_slots(const uint8_t *__restrict__ slots, uint32_t stride, uint64_t n, IndexedArgs a,
                uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    if (TM != kTabGlobal && TM != kTabFlat && TM != kTabFlat4) stage_table(a);
    const uint32_t lane = lane_id();
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t wave0 = uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t waves = uint64_t(gridDim.x) * wpb;
    const uint64_t step = waves * 64;
    constexpr bool RS = MODE == 4 || MODE == 5 || MODE == 6;  // lane-contiguous loads + permlane row swaps
    constexpr bool RSPF = MODE == 5;             // RS + the next batch's loads in flight (16 VGPRs)
    constexpr bool RSIN = MODE == 6;             // RS + the next batch's loads issued by the walk (pf below)
    constexpr bool COAL = MODE != 0 && !RS;      // lane-contiguous loads + quad DPP transpose
    constexpr bool NT = MODE >= 2;
    constexpr bool PF = MODE == 3;  // coalesced + next-batch register prefetch
    const uint32_t mine = COAL ? coal_packet(lane) : lane;  // packet of this lane within the batch
    // pulled batches: load mode 4 (the other modes prefetch the batch a grid stride ahead)
    BatchSource src;
    uint64_t base = src.first(MODE == 4 ? a.dyn : nullptr, n, a, wave0, waves);
    uint32_t d[16];
    u32x4 nv[4];
    if (!COAL && !RS && base < n) load16(slots + (base + lane < n ? base + lane : 0) * stride, d);
    if (PF && base + 64 <= n) load_coal<NT>(slots + base * 64, lane, nv);
    if ((RSPF || RSIN) && base + 64 <= n) load_rowswap<NT>(slots + base * 64, lane, nv);
    for (; base < n; base = src.next()) {
        const uint64_t idx = base + mine;
        const bool live = idx < n;
        const uint8_t *pkt = slots + (live ? idx : 0) * stride;
        uint32_t cur[16];
        if (RS) {
            if (base + 64 <= n) {
                u32x4 cv[4];
                if (RSIN) {  // this batch's loads were issued during the previous batch
                    rowswap_batch(nv, cur);
                } else {
                    if (RSPF) {
#pragma unroll
                        for (int j = 0; j < 4; ++j) cv[j] = nv[j];
                        const uint64_t nb = base + step;
                        if (nb + 64 <= n) load_rowswap<NT>(slots + nb * 64, lane, nv);
                    } else {
                        load_rowswap<NT>(slots + base * 64, lane, cv);
                    }
                    rowswap_batch(cv, cur);
                }
            } else {
                load16(pkt, cur);
            }
        } else if (COAL) {
            if (base + 64 <= n) {
                u32x4 cv[4];
                if (PF) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) cv[j] = nv[j];
                    const uint64_t nb = base + step;
                    if (nb + 64 <= n) load_coal<NT>(slots + nb * 64, lane, nv);
                } else {
                    load_coal<NT>(slots + base * 64, lane, cv);
                }
                transpose_batch(cv, lane, cur);
            } else {
                load16(pkt, cur);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; ++k) cur[k] = d[k];
            const uint64_t nb = base + step;
            if (nb < n) load16(slots + (nb + lane < n ? nb + lane : 0) * stride, d);  // prefetch
        }
        Fields f;
        // HYBRID walks: option ports from registers (as the frames kernels);
        // the streaming INDEXED kernel (C2) keeps the divergent far read:
        // it is VALU-bound, the select chain cost it 2.6 % (round 1), and
        // taking every option port from registers (no far read at all at
        // stride 64) 9 % (round 3, profiles/r3_ab/regports/)
        constexpr bool REG = TM == kTabFlatLds || TM == kTabFlatLds4 || TM == kTabFlatLds4U || TM == kTabFlatLdsG ||
                             TM == kTabFlatLdsP;
        parse_fields<REG, TM == kTabLdsNP>(cur, live, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
            far_dwords(pkt, stride, k, lo, hi);
        }, a.flags);
        const uint32_t res = classify_any<NS, TM>(a, f, [&] {
            if (RSIN) {
                const uint64_t nb = base + step;
                if (nb + 64 <= n) load_rowswap<NT>(slots + nb * 64, lane, nv);
            }
        });
        if (live && port_out) store_port<TM == kTabFlatLdsP>(port_out + idx, res);
        if (permit_out) {
            // permit bit p belongs to packet p: fetch packet `lane`'s verdict from the lane holding it
            const uint32_t src = COAL ? 4u * (lane & 15u) + (lane >> 4) : lane;
            const uint32_t r = COAL ? static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(
                                          static_cast<int>(src * 4), static_cast<int>(res)))
                                    : res;
            const uint64_t permit = ballot(base + lane < n && r != 0u);
            if (lane == 0) permit_out[base >> 6] = permit;
        }
    }
    src.finish(waves);
}

// (Round 3: compiled for 6 waves per SIMD — 80 VGPRs, a few spills — with
// two 768-thread workgroups per CU over 56-64 KB directories: C3 0.464 vs
// 0.463 ms, the extra waves bought back only what the smaller directories
// cost; profiles/r3_ab/c3_occupancy/)
template <int NS, int TM>
__global__ void __launch_bounds__(1024)
k_indexed_frames(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint64_t n,
                 IndexedArgs a, uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    if (TM != kTabGlobal && TM != kTabFlat && TM != kTabFlat4) stage_table(a);
    const uint32_t lane = lane_id();
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t waves = uint64_t(gridDim.x) * wpb;
    const uint64_t S = waves * 64;  // grid stride in packets
    const uint64_t wave0 = uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t base = wave0 * 64;
    auto desc_at = [&](uint64_t b) -> uint64_t {  // (branch-free, see load_frames_rs)
        return *(b + lane < n ? desc + b + lane : reinterpret_cast<const uint64_t *>(&g_zero16));
    };
    // classify the batch at b whose descriptor is ds and first 64 bytes d
    auto classify_batch = [&](uint64_t b, uint64_t ds, uint32_t(&d)[16]) {
        const bool live = b + lane < n;
        const uint32_t len = static_cast<uint32_t>(ds & 0xFFFFu);
        const uint8_t *pkt = frames + (ds >> 16);
        // bytes past the frame read as 0; IMIX frames are all >= 64 bytes, so
        // the clip is skipped unless some lane of the wave holds a shorter one
        if (ballot(live && len < 64u)) clip16(d, len);
        Fields f;
        parse_fields<true, TM == kTabLdsNP>(d, live, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
            far_dwords(pkt, len, k, lo, hi);
        }, a.flags);
        const uint32_t res = classify_any<NS, TM>(a, f, [] {});
        store_verdicts(b, lane, live, res, port_out, permit_out);
    };
    // Software pipeline.  Always: the next batch's descriptors load while this
    // batch is classified (the frame load depends on them).  PF (per-lane
    // HYBRID walks, whose LDS directories hold the CU to 16 waves and so leave
    // VGPRs to spare): also the next batch's 64-byte frame lines, into the
    // other of two register buffers (ping-pong, no copies), and the
    // descriptors of the batch after.
// (Round 6, VERDICT round 5 item 6, experiment builds NFFACL_EXP_FRAMES_PF:
// 1 = the next batch's frame lines in flight + descriptors two ahead, 2 =
// descriptors two batches ahead only — C3 0.4106 / 0.4157 and 0.4099 /
// 0.4065 vs 0.4127 / 0.4089 ms in alternating processes: within noise, the
// scattered frame reads still set the rate; profiles/r6_ab/c3pf/)
#ifndef NFFACL_EXP_FRAMES_PF
#define NFFACL_EXP_FRAMES_PF 0
#endif
    constexpr bool PF = TM == kTabSplit || (NFFACL_EXP_FRAMES_PF == 1 && TM == kTabFlatLds);  // (flat-LDS: +0.6 % on C3, profiles/r1_flat_lds/cold/)
    // (flat-LDS, round 2: one prefetch buffer with copies, 2 rounds — 124
    // VGPRs, no spill — ran 0.487 vs 0.469 ms on C3: the frame loads are not
    // what the walk waits on; profiles/r2_valu/pfab/.  Round 3: the same
    // prefetch issued from inside the walk, after the first window's entry
    // loads so that no entry wait queues behind it: 0.496 vs 0.473 ms,
    // profiles/r3_ab/)
    // Frame lines load cooperatively (load_frames_rs) and are assembled per
    // lane just before their batch is classified.
    auto run_batch = [&](uint64_t b, uint64_t ds, const u32x4(&v)[4]) {
        uint32_t d[16];
        rowswap_batch(v, d);
        classify_batch(b, ds, d);
    };
    if (PF) {
        if (base >= n) return;
        u32x4 A[4], B[4];
        uint64_t dsA = desc_at(base), dsB = 0;
        load_frames_rs(frames, dsA, lane, A);
        uint64_t dsN = desc_at(base + S);  // descriptor of the batch after the one in flight
        while (true) {
            const uint64_t b1 = base + S;
            if (b1 < n) {
                dsB = dsN;
                load_frames_rs(frames, dsB, lane, B);
                dsN = desc_at(b1 + S);
            }
            run_batch(base, dsA, A);
            if (b1 >= n) break;
            const uint64_t b2 = b1 + S;
            if (b2 < n) {
                dsA = dsN;
                load_frames_rs(frames, dsA, lane, A);
                dsN = desc_at(b2 + S);
            }
            run_batch(b1, dsB, B);
            if (b2 >= n) break;
            base = b2;
        }
    } else if (NFFACL_EXP_FRAMES_PF == 2 && !a.dyn) {  // experiment: descriptors two batches ahead (grid stride)
        uint64_t ds_next = desc_at(base), ds_next2 = desc_at(base + S);
        while (base < n) {
            const uint64_t ds = ds_next;
            u32x4 v[4];
            load_frames_rs(frames, ds, lane, v);
            ds_next = ds_next2;
            ds_next2 = desc_at(base + 2 * S);
            run_batch(base, ds, v);
            base += S;
        }
    } else {  // (pulled batches: BatchSource)
        BatchSource src;
        base = src.first(a.dyn, n, a, wave0, waves);
        uint64_t ds_next = desc_at(base);
        while (base < n) {
            const uint64_t ds = ds_next;
            u32x4 v[4];
            load_frames_rs(frames, ds, lane, v);
            const uint64_t nx = src.next();
            ds_next = desc_at(nx);  // issued after this batch's frame loads
            run_batch(base, ds, v);
            base = nx;
        }
        src.finish(waves);
    }
}

}  // namespace dev

// ---------------------------------------------------------------------------
// Host side of the engine
// ---------------------------------------------------------------------------

bool Tune::from_env(Tune &t, std::string &err) {
    t = Tune{};
    long v = 0;
    bool set = false;
    if (!env_knob("NFFACL_TUNE_COAL", 0, 6, v, set, err)) return false;
    if (set) t.coal = static_cast<int>(v);
    t.coal_set = set;
    if (!env_knob("NFFACL_TUNE_BLOCK", 64, 1024, v, set, err)) return false;
    if (set && v % 64 != 0) {
        err = "NFFACL_TUNE_BLOCK: expected a multiple of 64";
        return false;
    }
    if (set) t.block = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_PER_CU", 1, 32, v, set, err)) return false;
    if (set) t.per_cu = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_ROUNDS", 2, 4, v, set, err)) return false;
    if (set && v == 3) {
        err = "NFFACL_TUNE_ROUNDS: expected 2 or 4";
        return false;
    }
    if (set) t.rounds = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_LDS", 0, 1, v, set, err)) return false;
    if (set) t.lds = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DYN", 0, 2, v, set, err)) return false;
    if (set) t.dyn = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DYN_GMAX", 1, 64, v, set, err)) return false;
    if (set) t.dyn_gmax = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DYN_GMIN", 1, 64, v, set, err)) return false;
    if (set) t.dyn_gmin = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DYN_PULLS", 1, 64, v, set, err)) return false;
    if (set) t.dyn_pulls = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_DYN_TAIL", 1, 64, v, set, err)) return false;
    if (set) t.dyn_tail = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_PIPE", 0, 2, v, set, err)) return false;
    if (set) t.pipe = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_HOST_DMA", 0, 1, v, set, err)) return false;
    if (set) t.host_dma = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_HOST_BUFS", 2, nffacl_engine::kHostBufs, v, set, err)) return false;
    if (set) t.host_bufs = static_cast<int>(v);
    if (!env_knob("NFFACL_TUNE_HOST_CHUNK", 12, 24, v, set, err)) return false;
    if (set) t.host_chunk = static_cast<int>(v);
    return CompileOptions::from_env(t.copt, err);
}

// The scalar-call consumer's view of a compiled table (service.hpp): the
// forms the default compiler produces (LINEAR, INDEXED, HYBRID flat-LDS with
// positional slots); tuning-only forms get kSvcNone.
static SvcDesc service_desc(const CompiledTable &m) {
    SvcDesc d{};
    d.back = static_cast<uint32_t>(m.blob.size());
    d.dir8 = m.dir8;
    const FamilyIndex *fi[2] = {&m.idx4, &m.idx6};
    const uint32_t used = std::max(m.idx4.used_slots, m.idx6.used_slots);
    d.ns = used <= 2 ? 2u : used;
    if (m.algo == NFFACL_ALGO_LINEAR) {
        d.kind = kSvcLinear;
        d.off_rec4 = m.off_rec4;
        d.n4 = m.n4;
        d.off_rec6 = m.off_rec6;
        d.n6 = m.n6;
        return d;
    }
    const bool flat_lds = m.algo == NFFACL_ALGO_HYBRID && m.lds_dwords > 0 && m.idx4.entry_dwords == kHybEnt4Dwords;
    if ((d.ns > 4 && !flat_lds) || d.ns > kMaxSlots || m.slots_g || (m.algo == NFFACL_ALGO_HYBRID && !flat_lds))
        return d;  // kSvcNone
    d.kind = flat_lds ? kSvcFlat : kSvcIndexed;
    const uint32_t off_cold[2] = {m.off_rec4, m.off_rec6};
    for (int f = 0; f < 2; ++f) {
        SvcFamily &o = d.fam[f];
        o.off_resid = fi[f]->off_resid;
        o.n_resid = fi[f]->n_resid;
        o.off_cold = off_cold[f];
        o.off_ent_base = fi[f]->off_ent_base;
        for (uint32_t s = 0; s < kMaxSlots; ++s) {
            const DimInfo &di = fi[f]->dims[s];
            o.slot[s][0] = di.shift | di.shift2 << 8 | di.bits2 << 16;
            o.slot[s][1] = di.off_dir;
            o.slot[s][2] = di.off_ent;
            o.slot[s][3] = di.off_dir16;
        }
    }
    return d;
}

// Tables uploaded so far (DevTable::gen of the latest).
static std::atomic<uint32_t> g_table_epoch{0};

int compile_words(const nffacl_rules &rules, int algo, const CompileOptions &copt, DevTable &t,
                  std::vector<uint32_t> &words) {
    std::string err;
    if (!compile_table(rules, algo, copt, t.meta, err)) {
        set_last_error("compile: " + err);
        return NFFACL_ERR_INVALID_ARG;
    }
    const SvcDesc d = service_desc(t.meta);
    t.svc_kind = d.kind;
    words = t.meta.blob;
    words.resize(words.size() + kSvcDescDwords);
    std::memcpy(words.data() + t.meta.blob.size(), &d, sizeof d);
    return NFFACL_OK;
}

void table_resident(DevTable &t) {
    t.bytes = t.meta.blob.size() * sizeof(uint32_t);  // reported size: the table itself
    t.d_desc = t.d_blob + t.meta.blob.size();
    // the generation is drawn after the upload has completed (service.hip:
    // a consumer launched after the counter passed it sees the table)
    t.gen = g_table_epoch.fetch_add(1, std::memory_order_seq_cst) + 1;
}

int compile_upload(const nffacl_rules &rules, int algo, const CompileOptions &copt, TableHome &home, DevTable &t) {
    std::vector<uint32_t> words;
    const int st = compile_words(rules, algo, copt, t, words);
    if (st != NFFACL_OK) return st;
    const hipError_t e = t.upload(&home, words.data(), words.size());
    if (e != hipSuccess) {
        set_last_error(std::string("table upload: ") + hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? NFFACL_ERR_NOMEM : NFFACL_ERR_HIP;
    }
    table_resident(t);
    return NFFACL_OK;
}

uint32_t table_epoch() { return g_table_epoch.load(std::memory_order_seq_cst); }

int upload_table(nffacl_engine *eng, const nffacl_rules &rules, TablePtr &out) {
    auto t = std::make_shared<DevTable>();
    HIP_TRY(hipSetDevice(eng->device));
    const int st = compile_upload(rules, eng->algo_req, eng->tune.copt, eng->home, *t);
    if (st != NFFACL_OK) return st;
    out = std::move(t);
    return NFFACL_OK;
}

static uint32_t grid_for(const nffacl_engine *eng, uint64_t n, uint32_t block, uint32_t per_cu) {
    const uint64_t waves_needed = (n + 63) / 64;
    const uint64_t blocks_needed = (waves_needed * 64 + block - 1) / block;
    const uint64_t cap = uint64_t(eng->num_cus) * per_cu;
    return static_cast<uint32_t>(std::max<uint64_t>(1, std::min(blocks_needed, cap)));
}

// SlotField of a KeyKind (kernel key[] index).
static uint32_t field_of(uint32_t kind) {
    switch (kind) {
    case kKeyDst4: case kKeyDst6: return kFDst;
    case kKeySrc4: case kKeySrc6: return kFSrc;
    case kKeyDport: return kFDport;
    case kKeySport: return kFSport;
    default: return kFZero;
    }
}

static dev::IndexedArgs indexed_args(const DevTable *t) {
    dev::IndexedArgs a{};
    a.tab = t->d_blob;
    const bool hyb = t->meta.algo == NFFACL_ALGO_HYBRID;
    a.stage_dwords = hyb ? t->meta.lds_dwords : static_cast<uint32_t>(t->meta.blob.size());
    a.dir8 = hyb ? t->meta.dir8 : 0u;
    a.dir16 = hyb && (t->meta.idx4.dims[0].off_dir16 | t->meta.idx6.dims[0].off_dir16) != 0 ? 1u : 0u;
    a.generic = t->meta.slots_g ? 1u : 0u;
    auto fam = [&](const FamilyIndex &fi, uint32_t off_cold, dev::FamArgs &fa) {
        for (uint32_t k = 0; k < kMaxSlots; ++k) {
            const DimInfo &d = fi.dims[k];
            if (t->meta.slots_g && k >= fi.used_slots) {  // unused: key 0 into an empty directory
                fa.slot[k] = dev::SlotArgs{0, t->meta.off_empty_dir, 0, 0, kFZero, kFZero, 0, 0};
                continue;
            }
            // positional forms: slot k keys on field k ([dst, src, dport, sport]);
            // generalized slots (global-directory HYBRID): the fields compiled
            const uint32_t f1 = t->meta.slots_g ? field_of(d.kind) : k;
            const uint32_t f2 = t->meta.slots_g ? field_of(d.kind2) : uint32_t(kFZero);
            fa.slot[k] = dev::SlotArgs{d.shift, d.off_dir, d.off_ent, d.off_dir16, f1, f2, d.shift2, d.bits2};
        }
        fa.off_resid = fi.off_resid;
        fa.n_resid = fi.n_resid;
        fa.off_cold = off_cold;
        fa.off_ent_base = fi.off_ent_base;
    };
    fam(t->meta.idx4, t->meta.off_rec4, a.f4);
    fam(t->meta.idx6, t->meta.off_rec6, a.f6);
    a.off_params = hyb ? t->meta.off_params : 0u;
    a.live = 0;
    for (uint32_t k = 0; k < kMaxSlots; ++k)
        if (t->meta.slots_g || t->meta.idx4.dims[k].n_rules || t->meta.idx6.dims[k].n_rules) a.live |= 1u << k;
    return a;
}

// LDS budget per workgroup for a staged table (gfx950: 160 KiB per CU).
constexpr size_t kLdsBytes = 160 * 1024;

struct IndexedLaunch {
    int tm;  // dev::TableMode
    int ns;
    uint32_t block, per_cu;
    size_t lds_bytes;
};

// The kernel a table gets must match the layout it was compiled to: checked
// on the host before every indexed launch (a mismatch would read the blob
// with the wrong offsets).
static bool table_consistent(const DevTable *t) {
    const CompiledTable &m = t->meta;
    const size_t dw = m.blob.size();
    // entry numbers (and list offsets) stay below 2^23: the kernels scale
    // them with 24-bit multiplies (classify.hpp times_ew, classify_flat;
    // the window deltas multiply entry - candidate numbers as signed 24-bit)
    if (dw / kHybEnt4Dwords >= (size_t(1) << 23)) return false;
    if (m.algo == NFFACL_ALGO_HYBRID && (m.lds_dwords == 0 || m.idx4.entry_dwords == kHybEnt4Dwords))
        return m.idx4.entry_dwords == kHybEnt4Dwords && m.idx6.entry_dwords == kHybEnt6Dwords &&
               m.off_rec4 <= dw && m.off_rec6 <= dw &&
               size_t(m.lds_dwords) * sizeof(uint32_t) <= kHybLdsDirMaxBytes && m.lds_dwords <= dw &&
               // flat-LDS positional forms read their slot parameters from the staged image
               (m.lds_dwords == 0 || m.slots_g ||
                (m.off_params > 0 && m.off_params + kFlatParamDwords * kMaxSlots <= m.lds_dwords));
    if (m.algo == NFFACL_ALGO_HYBRID)
        return size_t(m.lds_dwords) * sizeof(uint32_t) <= kLdsTableBytes && m.lds_dwords <= dw &&
               m.idx4.entry_dwords == kEnt4Dwords && m.idx6.entry_dwords == kEnt6Dwords;
    return m.idx4.entry_dwords == kEnt4Dwords && m.idx6.entry_dwords == kEnt6Dwords;
}

// Widest table the pipelined walk takes.  (Round 5 held it at 6 slots: the
// NS = 7 kernel lost IPv6 matches.  Round 6 found why — a 64-bit shift
// reading its amount from the allocation's last VGPR sees the next wave's
// v0 on MI355X, tools/v127_probe.hip — removed the shift (classify.hpp
// hyb_miss) and checks every build for the pattern, tools/isa_guard.py.)
#ifndef NFFACL_PIPE_MAX_NS
#define NFFACL_PIPE_MAX_NS 8
#endif

// Launch shape of an indexed table; Tune overrides (frozen at engine creation).
static IndexedLaunch indexed_launch(const nffacl_engine *eng, const DevTable *t) {
    const Tune &tu = eng->tune;
    const uint32_t used = std::max(t->meta.idx4.used_slots, t->meta.idx6.used_slots);
    const int ns = used <= 2 ? 2 : static_cast<int>(used);
    IndexedLaunch L{dev::kTabGlobal, ns, 256u, 8u, 0};
    size_t staged = 0;
    // HYBRID: the compiled form decides (table.hpp) — lane form: directories
    // staged in LDS, inline entries walked per lane; flat form (lds_dwords 0):
    // directories and compact entries in global memory, candidates flat.
    if (t->meta.algo == NFFACL_ALGO_HYBRID && t->meta.lds_dwords == 0) {
        const bool r2 = tu.rounds == 2;
        L.tm = r2 ? dev::kTabFlat : dev::kTabFlat4;
        L.block = tu.block ? static_cast<uint32_t>(tu.block) : 256u;
        L.per_cu = tu.per_cu ? static_cast<uint32_t>(tu.per_cu) : 8u;
        L.lds_bytes = (r2 ? sizeof(dev::FlatScratch<2>) : sizeof(dev::FlatScratch<4>)) * (L.block / 64);
        return L;
    }
    if (t->meta.algo == NFFACL_ALGO_HYBRID && t->meta.idx4.entry_dwords == kHybEnt4Dwords) {  // flat-LDS
        L.block = tu.block ? static_cast<uint32_t>(tu.block) : 1024u;
        L.per_cu = tu.per_cu ? static_cast<uint32_t>(tu.per_cu) : 1u;
        const size_t image = size_t(t->meta.lds_dwords) * sizeof(uint32_t);
        const size_t lds4 = image + sizeof(dev::FlatScratch<4>) * (L.block / 64);
        const int rounds = tu.rounds ? tu.rounds : static_cast<int>(t->meta.flat_rounds);
        const bool r4 = rounds == 4 && lds4 <= kLdsBytes;
        L.tm = r4 ? (t->meta.flat_uncond ? dev::kTabFlatLds4U : dev::kTabFlatLds4) : dev::kTabFlatLds;
        L.lds_bytes = r4 ? lds4 : image + sizeof(dev::FlatScratch<2>) * (L.block / 64);
        if (t->meta.slots_g) {  // generalized slots: the generic kernel, always 4 rounds (its scratch)
            L.tm = dev::kTabFlatLdsG;
            L.lds_bytes = lds4;  // > kLdsBytes is refused by the launch check below
        } else if (tu.pipe && (t->meta.flat_uncond || tu.pipe == 2) && lds4 <= kLdsBytes && !tu.rounds &&
                   ns <= NFFACL_PIPE_MAX_NS &&
                   // its marks carry entry offsets in 23 bits (classify_flat_pipe)
                   t->meta.blob.size() / kHybEnt4Dwords < (size_t(1) << 22) - (size_t(1) << 16)) {
            // the pipelined walk (its scratch: FlatScratch<4>)
            L.tm = dev::kTabFlatLdsP;
            L.lds_bytes = lds4;
        }
        // (round 4: 2 workgroups per CU — one resident at a time, so that one
        // that starts late on a CU held by a resident consumer takes a
        // smaller share — ran C5 0.5810 / 0.5829 vs 0.5816 / 0.5736 ms alone
        // in two sweeps and +37 % instead of +81 % beside busy consumers; 4
        // per CU +18 %: profiles/r4_ab/grid/, r4_service/svc_overlap_*.  Kept
        // at one; NFFACL_TUNE_PER_CU=2-4 for GPUs shared with consumers.)
        return L;
    }
    if (t->meta.algo == NFFACL_ALGO_HYBRID) {
        staged = size_t(t->meta.lds_dwords) * sizeof(uint32_t);
        L.tm = dev::kTabSplit;
    } else {
        const size_t bytes = t->meta.blob.size() * sizeof(uint32_t);
        if (bytes <= kLdsTableBytes && tu.lds != 0) {
            L.tm = t->meta.ports_any ? dev::kTabLdsNP : dev::kTabLds;
            staged = bytes;
        }
    }
    if (L.tm != dev::kTabGlobal) {
        // 1024-thread workgroups: with twice the resident workgroups per CU
        // launched (below) C2 runs 0.2038-0.2057 vs 0.2142 ms with 768
        // (profiles/r5_ab/blocks/; round 3, one launch per resident slot,
        // 768 had won: 0.2119 vs 0.2161, profiles/r3_ab/blocks/)
        L.block = 1024u;
        // lane form: one workgroup per CU (its VGPRs allow no second one).
        // LDS-staged INDEXED: twice the workgroups that fit a CU at once
        // (two of 1024 threads), so that each takes half a share and one that
        // starts late (its CU's LDS held by a resident consumer, §4.7) adds
        // half the tail: C2 0.2145 vs 0.2200 ms alone (profiles/r5_ab/pcu/)
        L.per_cu = L.tm == dev::kTabSplit
                       ? 1u
                       : 2u * static_cast<uint32_t>(
                                  std::max<size_t>(1, std::min<size_t>(2, kLdsBytes / std::max<size_t>(staged, 16))));
        L.lds_bytes = std::max<size_t>(staged, 16);
    }
    if (tu.block) L.block = static_cast<uint32_t>(tu.block);
    if (tu.per_cu) L.per_cu = static_cast<uint32_t>(tu.per_cu);
    return L;
}

template <class K>
static hipError_t allow_lds(K kernel) {
    return hipFuncSetAttribute(reinterpret_cast<const void *>(kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kLdsBytes));
}

// Load modes (64-byte slots): 0 one row per lane (+ next-batch register
// prefetch; any stride); 1 lane-contiguous + quad DPP transpose; 2 = 1 with
// non-temporal loads; 3 = 2 + register prefetch; 4 lane-contiguous
// non-temporal + permlane row-swap transpose (default).  Interleaved A/B in
// one process (profiles/r1_ab/): mode 4 0.2195 ms, 2 0.2203, 0 0.2475 (C2).
// Modes 1-3 are built for the LDS-staged table only (the A/B experiments).
template <int NS, int TM>
static hipError_t allow_lds_modes() {
    hipError_t e = allow_lds(dev::k_indexed_slots<NS, TM, 0>);
    if (e == hipSuccess) e = allow_lds(dev::k_indexed_slots<NS, TM, 4>);
    if (TM == dev::kTabFlatLds || TM == dev::kTabFlatLds4 || TM == dev::kTabFlatLds4U || TM == dev::kTabFlatLdsG ||
        TM == dev::kTabFlatLdsP)
        if (e == hipSuccess) e = allow_lds(dev::k_indexed_slots<NS, TM, 5>);
    if constexpr (TM == dev::kTabFlatLdsP)
        if (e == hipSuccess) e = allow_lds(dev::k_indexed_slots<NS, TM, 6>);
    if (TM == dev::kTabLds) {
        if (e == hipSuccess) e = allow_lds(dev::k_indexed_slots<NS, dev::kTabLds, 1>);
        if (e == hipSuccess) e = allow_lds(dev::k_indexed_slots<NS, dev::kTabLds, 2>);
        if (e == hipSuccess) e = allow_lds(dev::k_indexed_slots<NS, dev::kTabLds, 3>);
    }
    if (e == hipSuccess) e = allow_lds(dev::k_indexed_frames<NS, TM>);
    return e;
}

// Calls f(integral_constant<NS>, integral_constant<TM>) for the runtime pair.
template <class F>
static void dispatch_indexed(int ns, int tm, F &&f) {
#ifdef NFFACL_PROBE_NS  // register / ISA probe builds only (make probe): one slot count, two flat walks
    (void)ns;
    if (tm == dev::kTabFlatLdsP) f(std::integral_constant<int, NFFACL_PROBE_NS>{}, std::integral_constant<int, dev::kTabFlatLdsP>{});
    else f(std::integral_constant<int, NFFACL_PROBE_NS>{}, std::integral_constant<int, dev::kTabFlatLds4U>{});
#else
    auto with_ns = [&](auto nsc) {
        switch (tm) {
        case dev::kTabLds: f(nsc, std::integral_constant<int, dev::kTabLds>{}); break;
        case dev::kTabLdsNP: f(nsc, std::integral_constant<int, dev::kTabLdsNP>{}); break;
        case dev::kTabSplit: f(nsc, std::integral_constant<int, dev::kTabSplit>{}); break;
        case dev::kTabFlat: f(nsc, std::integral_constant<int, dev::kTabFlat>{}); break;
        case dev::kTabFlat4: f(nsc, std::integral_constant<int, dev::kTabFlat4>{}); break;
        case dev::kTabFlatLds: f(nsc, std::integral_constant<int, dev::kTabFlatLds>{}); break;
        case dev::kTabFlatLds4: f(nsc, std::integral_constant<int, dev::kTabFlatLds4>{}); break;
        case dev::kTabFlatLds4U: f(nsc, std::integral_constant<int, dev::kTabFlatLds4U>{}); break;
        case dev::kTabFlatLdsG: f(nsc, std::integral_constant<int, dev::kTabFlatLdsG>{}); break;
        case dev::kTabFlatLdsP: f(nsc, std::integral_constant<int, dev::kTabFlatLdsP>{}); break;
        default: f(nsc, std::integral_constant<int, dev::kTabGlobal>{}); break;
        }
    };
    // generalized slots (global-directory flat kernels only): up to kMaxSlots
    auto with_ns_flat = [&](auto nsc) {
        switch (tm) {
        case dev::kTabFlat: f(nsc, std::integral_constant<int, dev::kTabFlat>{}); break;
        case dev::kTabFlatLds: f(nsc, std::integral_constant<int, dev::kTabFlatLds>{}); break;
        case dev::kTabFlatLds4: f(nsc, std::integral_constant<int, dev::kTabFlatLds4>{}); break;
        case dev::kTabFlatLds4U: f(nsc, std::integral_constant<int, dev::kTabFlatLds4U>{}); break;
        case dev::kTabFlatLdsG: f(nsc, std::integral_constant<int, dev::kTabFlatLdsG>{}); break;
        case dev::kTabFlatLdsP: f(nsc, std::integral_constant<int, dev::kTabFlatLdsP>{}); break;
        default: f(nsc, std::integral_constant<int, dev::kTabFlat4>{}); break;
        }
    };
    if (ns == 2) with_ns(std::integral_constant<int, 2>{});
    else if (ns == 3) with_ns(std::integral_constant<int, 3>{});
    else if (ns == 4) with_ns(std::integral_constant<int, 4>{});
    else if (ns == 5) with_ns_flat(std::integral_constant<int, 5>{});
    else if (ns == 6) with_ns_flat(std::integral_constant<int, 6>{});
    else if (ns == 7) with_ns_flat(std::integral_constant<int, 7>{});
    else with_ns_flat(std::integral_constant<int, 8>{});
#endif
}

int prepare_kernels() {
    static std::once_flag once;
    static hipError_t err = hipSuccess;
    std::call_once(once, [] {
        for (int ns = 2; ns <= int(kMaxSlots); ++ns)
            for (int tm : {int(dev::kTabLds), int(dev::kTabLdsNP), int(dev::kTabSplit), int(dev::kTabFlatLds), int(dev::kTabFlatLds4),
                           int(dev::kTabFlatLds4U), int(dev::kTabFlatLdsG), int(dev::kTabFlatLdsP)}) {
                if (ns > 4 && tm != dev::kTabFlatLds && tm != dev::kTabFlatLds4 && tm != dev::kTabFlatLds4U &&
                    tm != dev::kTabFlatLdsG && tm != dev::kTabFlatLdsP)
                    continue;  // flat walks only
                dispatch_indexed(ns, tm, [&](auto nsc, auto tmc) {
                    const hipError_t e = allow_lds_modes<decltype(nsc)::value, decltype(tmc)::value>();
                    if (e != hipSuccess) err = e;
                });
            }
    });
    if (err != hipSuccess) {
        set_last_error(std::string("hipFuncSetAttribute(LDS): ") + hipGetErrorString(err));
        return NFFACL_ERR_HIP;
    }
    return NFFACL_OK;
}

// The pull heads of launches on `stream` (nullptr: none free, grid stride).
// A head block is reused by the next launch on the same handle, so the
// handle must name ONE ordered stream and the launch must run when it is
// enqueued: hipStreamPerThread names a different stream on every thread, and
// a launch captured into a graph may be replayed beside another launch on
// the same stream — both take the grid stride.
static uint32_t *dyn_heads(nffacl_engine *eng, hipStream_t stream) {
    if (!eng->d_dyn || stream == hipStreamPerThread) return nullptr;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(stream, &cs) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (cs != hipStreamCaptureStatusNone) return nullptr;
    std::lock_guard<std::mutex> g(eng->dyn_mu);
    for (int i = 0; i < eng->dyn_used; ++i)
        if (eng->dyn_stream[i] == stream) return eng->d_dyn + size_t(i) * kDynBlockWords;
    if (eng->dyn_used == nffacl_engine::kDynStreams) return nullptr;
    eng->dyn_stream[eng->dyn_used] = stream;
    return eng->d_dyn + size_t(eng->dyn_used++) * kDynBlockWords;
}

// Pulled batches for a launch of `grid` workgroups of `block` threads over n
// packets: pulls of up to ~1/4 of a wave's share (at most 16 batches), so
// that the heads see a few pulls per wave (one head saturates near 88
// pulls per microsecond: MI355X_MICROARCH.md, dequeue).
static void dyn_args(nffacl_engine *eng, hipStream_t stream, uint32_t grid, uint32_t block, uint64_t n,
                     dev::IndexedArgs &a) {
    a.dyn = dyn_heads(eng, stream);
    const uint64_t waves = uint64_t(grid) * (block / 64), nb = (n + 63) / 64;
    const Tune &tu = eng->tune;
    a.dyn_g = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(tu.dyn_gmax, nb / (waves * tu.dyn_pulls))));
    a.dyn_gmin = std::min<uint32_t>(a.dyn_g, static_cast<uint32_t>(tu.dyn_gmin));
    a.dyn_wpx = static_cast<uint32_t>(std::max<uint64_t>(1, waves * tu.dyn_tail / 16));
}

// Load mode of a slots launch: long flat walks (kTabFlatLds4U, C5) default
// to mode 5, the next batch's packets in flight: 0.6278 / 0.6312 vs 0.6340 /
// 0.6328 ms (profiles/r3_ab/c5_mode5/); everything else to mode 4.
static int slots_mode(const nffacl_engine *eng, const IndexedLaunch &L, uint32_t stride) {
    int mode = stride == 64 ? eng->tune.coal : 0;
    if (stride == 64 && !eng->tune.coal_set && (L.tm == dev::kTabFlatLds4U || L.tm == dev::kTabFlatLdsG)) mode = 5;
    return mode;
}

static bool flat_lds_walk(int tm) {
    return tm == dev::kTabFlatLds || tm == dev::kTabFlatLds4 || tm == dev::kTabFlatLds4U || tm == dev::kTabFlatLdsG ||
           tm == dev::kTabFlatLdsP;
}

// Pulled batches (BatchSource): the flat-LDS walks (C5: 0.5111 vs 0.5341 ms
// alone with pulls of 12-16 batches — 0.5159 / 0.5208 / 0.5247 with at
// least 8 / 16 / 4 — and +9-13 % instead of +80 % beside busy consumers,
// profiles/r5_ab/dyn/); not the short per-lane walks (C2 0.316 vs 0.220 ms:
// its waves pull in lockstep and wait on the heads, and a wave's chunk of
// consecutive batches spreads its group's loads over 10x the pages of the
// grid stride: 0.27 ms with one pull per wave; profiles/r5_ab/dyn/).
static bool slots_pull(const nffacl_engine *eng, const IndexedLaunch &L, int mode) {
    return mode == 4 && (eng->tune.dyn == 2 || (eng->tune.dyn == 1 && flat_lds_walk(L.tm)));
}

template <int NS, int TM>
static void launch_slots_tm(int mode, const IndexedLaunch &L, uint32_t grid, hipStream_t stream,
                            const uint8_t *d_slots, uint32_t stride, uint64_t n, const dev::IndexedArgs &a,
                            uint32_t *d_port, uint64_t *d_permit) {
    const dim3 g(grid), b(L.block);
    const size_t lds = TM == dev::kTabGlobal ? 0 : L.lds_bytes;
    if constexpr (TM == dev::kTabFlatLds || TM == dev::kTabFlatLds4 || TM == dev::kTabFlatLds4U ||
                  TM == dev::kTabFlatLdsG || TM == dev::kTabFlatLdsP) {  // load modes 0, 4, 5
        if constexpr (TM == dev::kTabFlatLdsP) {  // mode 6: the walk issues the next batch's loads
            if (mode == 6) {
                hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 6>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
                return;
            }
        }
        if (mode == 0)
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 0>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
        else if (mode == 5)
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 5>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
        else
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 4>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
    } else if constexpr (TM != dev::kTabLds) {  // built with load modes 0 and 4 only
        if (mode == 0)
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 0>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
        else
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 4>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
    } else if (mode >= 1 && mode <= 3) {
        if (mode == 1)
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, dev::kTabLds, 1>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
        else if (mode == 2)
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, dev::kTabLds, 2>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
        else
            hipLaunchKernelGGL((dev::k_indexed_slots<NS, dev::kTabLds, 3>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
    } else if (mode == 0) {
        hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 0>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
    } else {
        hipLaunchKernelGGL((dev::k_indexed_slots<NS, TM, 4>), g, b, lds, stream, d_slots, stride, n, a, d_port, d_permit);
    }
}

template <int NS, int TM>
static void launch_frames_tm(const IndexedLaunch &L, uint32_t grid, hipStream_t stream, const uint8_t *d_frames,
                             const uint64_t *d_desc, uint64_t n, const dev::IndexedArgs &a, uint32_t *d_port,
                             uint64_t *d_permit) {
    const size_t lds = TM == dev::kTabGlobal ? 0 : L.lds_bytes;
    hipLaunchKernelGGL((dev::k_indexed_frames<NS, TM>), dim3(grid), dim3(L.block), lds, stream, d_frames, d_desc, n,
                       a, d_port, d_permit);
}

int launch_slots(nffacl_engine *eng, DevTable *t, const uint8_t *d_slots, uint32_t stride,
                 uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream, uint32_t flags) {
    if (n == 0) return NFFACL_OK;
    if (t->meta.algo != NFFACL_ALGO_LINEAR) {
        if (!table_consistent(t)) {
            set_last_error("compiled table layout does not match its kernel");
            return NFFACL_ERR_INVALID_ARG;
        }
        dev::IndexedArgs a = indexed_args(t);
        a.flags = flags;
        const IndexedLaunch L = indexed_launch(eng, t);
        if (L.lds_bytes > kLdsBytes) {  // (a generalized-slot table with a directory image too large for its scratch)
            set_last_error("compiled table's LDS image and scratch exceed the CU's LDS");
            return NFFACL_ERR_INVALID_ARG;
        }
        const uint32_t grid = grid_for(eng, n, L.block, L.per_cu);
        const int mode = slots_mode(eng, L, stride);
        if (slots_pull(eng, L, mode)) dyn_args(eng, stream, grid, L.block, n, a);
        // (the pipelined walk: load mode 4 — mode 6, the next batch's loads
        // issued from inside the walk, spilled and ran 0.64 vs 0.53 ms on C5:
        // NFFACL_TUNE_COAL=6, profiles/r5_ab/)
        dispatch_indexed(L.ns, L.tm, [&](auto nsc, auto tmc) {
            launch_slots_tm<decltype(nsc)::value, decltype(tmc)::value>(mode, L, grid, stream, d_slots, stride, n, a,
                                                                      d_port, d_permit);
        });
    } else {
        const uint32_t block = 256;
        dev::LinearArgs a{t->d_blob + t->meta.off_rec4, t->meta.n4, t->d_blob + t->meta.off_rec6,
                          t->meta.n6, flags};
        const uint32_t grid = grid_for(eng, n, block, 8);
        hipLaunchKernelGGL(dev::k_linear_slots, dim3(grid), dim3(block), 0, stream, d_slots, stride,
                           n, a, d_port, d_permit);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(t->note_use(stream));
    return NFFACL_OK;
}

int launch_frames(nffacl_engine *eng, DevTable *t, const uint8_t *d_frames,
                  const uint64_t *d_desc, uint64_t n, uint32_t *d_port, uint64_t *d_permit,
                  hipStream_t stream, uint32_t flags) {
    if (n == 0) return NFFACL_OK;
    if (t->meta.algo != NFFACL_ALGO_LINEAR) {
        if (!table_consistent(t)) {
            set_last_error("compiled table layout does not match its kernel");
            return NFFACL_ERR_INVALID_ARG;
        }
        dev::IndexedArgs a = indexed_args(t);
        a.flags = flags;
        const IndexedLaunch L = indexed_launch(eng, t);
        if (L.lds_bytes > kLdsBytes) {  // (a generalized-slot table with a directory image too large for its scratch)
            set_last_error("compiled table's LDS image and scratch exceed the CU's LDS");
            return NFFACL_ERR_INVALID_ARG;
        }
        const uint32_t grid = grid_for(eng, n, L.block, L.per_cu);
        // (pulled batches: C3 0.442 vs 0.396 ms; NFFACL_TUNE_DYN=2 only)
        if (L.tm != dev::kTabSplit && eng->tune.dyn == 2) dyn_args(eng, stream, grid, L.block, n, a);
        dispatch_indexed(L.ns, L.tm, [&](auto nsc, auto tmc) {
            launch_frames_tm<decltype(nsc)::value, decltype(tmc)::value>(L, grid, stream, d_frames, d_desc, n, a,
                                                                       d_port, d_permit);
        });
    } else {
        const uint32_t block = 256;
        dev::LinearArgs a{t->d_blob + t->meta.off_rec4, t->meta.n4, t->d_blob + t->meta.off_rec6,
                          t->meta.n6, flags};
        const uint32_t grid = grid_for(eng, n, block, 8);
        hipLaunchKernelGGL(dev::k_linear_frames, dim3(grid), dim3(block), 0, stream, d_frames, d_desc,
                           n, a, d_port, d_permit);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(t->note_use(stream));
    return NFFACL_OK;
}

// The kernel the active table's 64-byte-slot launches take (ABI 7,
// nffacl_engine_kernel_info): tests assert which walk ran.
int slots_kernel_info(nffacl_engine *eng, nffacl_kernel_info *out) {
    const TablePtr t = acquire_table(eng);
    if (!t) return NFFACL_ERR_INVALID_ARG;
    *out = nffacl_kernel_info{};
    if (t->meta.algo == NFFACL_ALGO_LINEAR) {
        out->walk = NFFACL_WALK_LINEAR;
        out->block = 256;
        out->per_cu = 8;
        return NFFACL_OK;
    }
    const IndexedLaunch L = indexed_launch(eng, t.get());
    switch (L.tm) {
    case dev::kTabLds: case dev::kTabLdsNP: out->walk = NFFACL_WALK_INDEXED_LDS; break;
    case dev::kTabSplit: out->walk = NFFACL_WALK_HYBRID_LANE; break;
    case dev::kTabFlat: case dev::kTabFlat4: out->walk = NFFACL_WALK_FLAT; break;
    case dev::kTabFlatLds: case dev::kTabFlatLds4: case dev::kTabFlatLds4U: out->walk = NFFACL_WALK_FLAT_LDS; break;
    case dev::kTabFlatLdsG: out->walk = NFFACL_WALK_FLAT_LDS_GENERIC; break;
    case dev::kTabFlatLdsP: out->walk = NFFACL_WALK_FLAT_LDS_PIPELINED; break;
    default: out->walk = NFFACL_WALK_INDEXED_GLOBAL; break;
    }
    out->slots = static_cast<uint32_t>(L.ns);
    out->rounds = L.tm == dev::kTabFlat || L.tm == dev::kTabFlatLds ? 2u : flat_lds_walk(L.tm) || L.tm == dev::kTabFlat4 ? 4u : 0u;
    out->block = L.block;
    out->per_cu = L.per_cu;
    out->lds_bytes = L.lds_bytes;
    out->load_mode = slots_mode(eng, L, 64);
    out->pulled = slots_pull(eng, L, out->load_mode) && eng->d_dyn ? 1 : 0;
    return NFFACL_OK;
}

}  // namespace nffacl
