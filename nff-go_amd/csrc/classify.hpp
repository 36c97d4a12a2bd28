// classify.hpp — device-side parse + match helpers of libnffacl (internal),
// shared by the batch kernels (engine.hip) and the persistent scalar-call
// consumer (service.hip).  See engine.hip for the execution model.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "devutil.hpp"
#include "nffacl.h"
#include "table.hpp"

namespace nffacl {
namespace dev {

// 16 zero bytes in global memory: the load address of a lane with nothing
// to read, so that loads need no per-lane branch.
static __device__ u32x4 g_zero16 = {0u, 0u, 0u, 0u};

__device__ __forceinline__ uint32_t funnel16(uint32_t hi, uint32_t lo) {
    // ({hi,lo} >> 16)[31:0] : wire bytes 4k+2 .. 4k+5 as a LE dword
    return __builtin_amdgcn_alignbit(hi, lo, 16);
}

// Byte-swap each 16-bit half: LE dword of wire bytes [p0 p1 p2 p3] ->
// (p0<<8|p1) | (p2<<8|p3) << 16 = sport | dport << 16 (SwapBytesUint16,
// packet/packet.go:713-715, applied by l4ACL acl.go:511, 515).
__device__ __forceinline__ uint32_t swap_halves(uint32_t w) {
    return __builtin_amdgcn_perm(w, w, 0x02030001u);  // one v_perm: bytes 1 0 3 2
}

// Non-zero iff some port of `ports` (sport | dport << 16) is outside
// [lo, hi] per half (l4ACL, acl.go:512-518).
__device__ __forceinline__ uint32_t port_miss(uint32_t ports, uint32_t lo, uint32_t hi) {
    u16x2 p = __builtin_bit_cast(u16x2, ports);
    u16x2 l = __builtin_bit_cast(u16x2, lo);
    u16x2 h = __builtin_bit_cast(u16x2, hi);
    u16x2 c = __builtin_elementwise_min(__builtin_elementwise_max(p, l), h);
    return __builtin_bit_cast(uint32_t, c) ^ ports;
}

// Header fields of one packet (Appendix A of SURVEY.md).
struct Fields {
    bool is4, is6;
    uint32_t proto;
    uint32_t ports;     // sport | dport << 16 (host order)
    uint32_t s[4], t[4];  // src / dst words (IPv4 uses [0])
};

// Parse the header fields from the first 64 bytes (d[0..15]) of a packet.
// `far(k)` returns the little-endian dwords k and k+1 of the packet (bytes past
// the slot/frame end as 0) for the rare IPv4 header whose IHL != 5 puts the L4
// ports somewhere other than bytes 34..37; it runs in a divergent branch that
// only lanes with IP options take.
// `vlan` (wave-uniform launch flag NFFACL_PARSE_VLAN) selects
// ParseAllKnownL3CheckVLAN (packet/vlan.go:104-117) over ParseAllKnownL3: a
// frame whose EtherType is 0x8100 has its L3 header 4 bytes (one dword) later
// and the tag's EtherType decides the family, so a tagged lane shifts d[3..14]
// down by one dword and parses as usual (d[15] is never read afterwards).
// REG_OPTS (frames kernels): ports that lie inside the 64 bytes in registers
// (IHL <= 11, untagged) come from them through a select chain, so only lanes
// whose ports lie past byte 64 read memory — most waves of C3 have some lane
// with options, and its dependent far read stalled the whole wave.
// NOPORTS: the caller's table tests no port; f.ports is left 0 and no
// option-port dword is read.
template <bool REG_OPTS = false, bool NOPORTS = false, class FarDwords>
__device__ __forceinline__ void parse_fields(uint32_t (&d)[16], bool live, Fields &f, FarDwords far,
                                             uint32_t flags) {
    const bool vlan = (flags & NFFACL_PARSE_VLAN) != 0;
    uint32_t l3dw = 3u;  // dword holding the first L3 byte (at byte 2 of it)
    if (vlan) {
        const bool tagged = (d[3] & 0xFFFFu) == 0x0081u;  // 0x8100 on the wire
        if (ballot(tagged)) {
#pragma unroll
            for (int k = 3; k < 15; ++k) d[k] = tagged ? d[k + 1] : d[k];
            l3dw = tagged ? 4u : 3u;
        }
    }
    // ParseAllKnownL3: EtherType at wire bytes 12-13 (packet.go:238-243, 264-269)
    const uint32_t et = d[3] & 0xFFFFu;
    f.is4 = live && et == 0x0008u;  // 0x0800 on the wire
    f.is6 = live && et == 0xDD86u;  // 0x86DD on the wire
    // IPv4: proto byte 23, src 26..29, dst 30..33, L4 at 14 + 4*IHL (packet.go:278-280)
    // IPv6: proto byte 20, src 22..37, dst 38..53, L4 at 54 (packet.go:283-285)
    const uint32_t ihl = (d[3] >> 16) & 0xFu;
    uint32_t pw = f.is6 ? funnel16(d[14], d[13]) : funnel16(d[9], d[8]);
    if (NOPORTS) {
        pw = 0u;
    } else if (REG_OPTS) {
        const bool opt = f.is4 && ihl != 5u;
        if (ballot(opt)) {
            // in the (VLAN-shifted) registers the L4 dword is 3 + IHL; valid
            // through d[15] untagged, d[14] tagged (d[15] is stale there)
            const uint32_t k = 3u + ihl, lim = 15u - (l3dw - 3u);
            uint32_t lo = 0, hi = 0;
#pragma unroll
            for (uint32_t j = 8; j <= 14; ++j) {
                lo = k == j ? d[j] : lo;
                hi = k == j ? d[j + 1] : hi;
            }
            if (opt) pw = funnel16(hi, lo);
            if (opt && (k + 1u > lim || k < 8u)) {  // past the registers, or a malformed IHL < 5
                far(l3dw + ihl, lo, hi);
                pw = funnel16(hi, lo);
            }
        }
    } else if (f.is4 && ihl != 5u) {
        // L4 bytes L3+4*IHL .. +3 = dword l3dw+IHL, byte 2.  (Taking IHL <= 11
        // from the registers instead, through a select chain, measured 2.6 %
        // slower on C2 and 1 % faster on C5 in one-process A/B: memory.)
        uint32_t lo, hi;
        far(l3dw + ihl, lo, hi);
        pw = funnel16(hi, lo);
    }
    f.ports = swap_halves(pw);
    f.proto = f.is6 ? (d[5] & 0xFFu) : (d[5] >> 24);
    // Address words without a branch: wire dwords F(k) = bytes 4k+2..4k+5
    // for k = 5..12 serve both families (IPv4 src = F6, dst = F7; IPv6 src =
    // F5..F8, dst = F9..F12).  Words 1..3 are meaningful for IPv6 lanes only
    // (every consumer reads them for IPv6 packets alone).
    uint32_t F[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) F[k] = funnel16(d[6 + k], d[5 + k]);
    f.s[0] = f.is6 ? F[0] : F[1];
    f.t[0] = f.is6 ? F[4] : F[2];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        f.s[k] = F[k];
        f.t[k] = F[4 + k];
    }
}

// Dwords k and k+1 of a packet whose readable, zero-padded extent is `lim`
// bytes from `base` (4-byte aligned); bytes at or past `lim` read as 0.
__device__ __forceinline__ void far_dwords(const uint8_t *base, uint32_t lim, uint32_t k,
                                           uint32_t &lo, uint32_t &hi) {
    // both dwords loaded together, without a branch (a dword wholly past the
    // extent is read from the zero block): one round trip, not two
    const uint32_t *p = reinterpret_cast<const uint32_t *>(base);
    const uint32_t *z = reinterpret_cast<const uint32_t *>(&g_zero16);
    const int r0 = static_cast<int>(lim) - static_cast<int>(4 * k), r1 = r0 - 4;
    const uint32_t v0 = *(r0 > 0 ? p + k : z), v1 = *(r1 > 0 ? p + k + 1 : z);
    auto keep = [](int rem) -> uint32_t { return rem >= 4 ? 0xFFFFFFFFu : rem <= 0 ? 0u : (1u << (8 * rem)) - 1u; };
    lo = v0 & keep(r0);
    hi = v1 & keep(r1);
}

// LINEAR: first-match scan in rule order, wave-uniform records.
__device__ __forceinline__ uint32_t classify_linear(const Fields &f,
                                                     const uint32_t *__restrict__ rec4, uint32_t n4,
                                                     const uint32_t *__restrict__ rec6, uint32_t n6) {
    uint32_t res = 0;
    bool pend = f.is4;
    if (ballot(pend)) {
        for (uint32_t r = 0; r < n4; ++r) {
            const uint32_t *R = rec4 + r * kRec4Dwords;
            uint32_t m = ((f.s[0] ^ R[0]) & R[1]) | ((f.t[0] ^ R[2]) & R[3]);
            const uint32_t meta = R[4];
            const uint32_t idm = (meta >> 8) & 0xFFu;
            if (idm) m |= (f.proto ^ meta) & idm;
            if (meta & kMetaPortCheck) m |= port_miss(f.ports, R[5], R[6]);
            const bool take = pend && m == 0u;
            if (ballot(take)) {
                if (take) { res = R[7]; pend = false; }
                if (!ballot(pend)) break;
            }
        }
    }
    pend = f.is6;
    if (ballot(pend)) {
        for (uint32_t r = 0; r < n6; ++r) {
            const uint32_t *R = rec6 + r * kRec6Dwords;
            uint32_t m = ((f.s[0] ^ R[0]) & R[4]) | ((f.s[1] ^ R[1]) & R[5]) |
                         ((f.s[2] ^ R[2]) & R[6]) | ((f.s[3] ^ R[3]) & R[7]) |
                         ((f.t[0] ^ R[8]) & R[12]) | ((f.t[1] ^ R[9]) & R[13]) |
                         ((f.t[2] ^ R[10]) & R[14]) | ((f.t[3] ^ R[11]) & R[15]);
            const uint32_t meta = R[16];
            const uint32_t idm = (meta >> 8) & 0xFFu;
            if (idm) m |= (f.proto ^ meta) & idm;
            if (meta & kMetaPortCheck) m |= port_miss(f.ports, R[17], R[18]);
            const bool take = pend && m == 0u;
            if (ballot(take)) {
                if (take) { res = R[19]; pend = false; }
                if (!ballot(pend)) break;
            }
        }
    }
    return res;
}

// Dense slots: packet i at slots + i*stride; the first 64 bytes are loaded
// with four 16-byte loads.  Plain loads, not non-temporal: with one lane per
// 64-byte row every cache line is consumed by four successive instructions,
// and the nt policy cost 30% of stream bandwidth on this pattern
// (profiles/r1_sol/sol.out: rows 5.26 TB/s vs rows_nt 3.66 TB/s).
__device__ __forceinline__ void load16(const uint8_t *__restrict__ p, uint32_t (&d)[16]) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const u32x4 v = q[j];
        d[4 * j + 0] = v.x;
        d[4 * j + 1] = v.y;
        d[4 * j + 2] = v.z;
        d[4 * j + 3] = v.w;
    }
}

// ---- lane-contiguous ("coalesced") batch load for 64-byte slots ------------
//
// A wave's 64 packets are 4 KiB contiguous.  Instruction j loads KiB j with
// lane l taking 16 bytes: packet 16j + l/4, chunk l%4 — every instruction
// reads 1 KiB contiguous (the fastest HBM pattern measured: sol `coalesced`
// 5.9 TB/s vs 5.3 TB/s for one 64-byte row per lane).  A 4x4 transpose inside
// each lane quad (two DPP butterfly stages per dword plane) then gives lane
// l = 4q + i all four chunks of packet 16i + q.

template <bool NT>
__device__ __forceinline__ void load_coal(const uint8_t *__restrict__ wave_base, uint32_t lane, u32x4 (&v)[4]) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(wave_base) + lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = NT ? __builtin_nontemporal_load(q + 64 * j) : q[64 * j];
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t x) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), CTRL, 0xF, 0xF, false));
}

// v[k] = value of instruction k in this lane; returns f[c] = quad-mate c's
// value of instruction (lane & 3).  Each butterfly stage sends one select per
// pair and receives it with one unconditional DPP move whose result feeds both
// arms of the following selects — a DPP result used in only one arm gets sunk
// into a divergent branch, where it reads inactive lanes.
__device__ __forceinline__ void quad_transpose(const uint32_t (&v)[4], uint32_t (&f)[4], bool b0, bool b1) {
    constexpr int kSwap1 = 0xB1;  // quad_perm [1,0,3,2]
    constexpr int kSwap2 = 0x4E;  // quad_perm [2,3,0,1]
    const uint32_t r0 = dpp<kSwap1>(b0 ? v[0] : v[1]);
    const uint32_t r1 = dpp<kSwap1>(b0 ? v[2] : v[3]);
    uint32_t s[4];
    s[0] = b0 ? r0 : v[0];
    s[1] = b0 ? v[1] : r0;
    s[2] = b0 ? r1 : v[2];
    s[3] = b0 ? v[3] : r1;
    const uint32_t q0 = dpp<kSwap2>(b1 ? s[0] : s[2]);
    const uint32_t q1 = dpp<kSwap2>(b1 ? s[1] : s[3]);
    f[0] = b1 ? q0 : s[0];
    f[1] = b1 ? q1 : s[1];
    f[2] = b1 ? s[2] : q0;
    f[3] = b1 ? s[3] : q1;
}

// Rebuild this lane's packet (d[16] = its first 64 bytes) from the 4 loads.
__device__ __forceinline__ void transpose_batch(const u32x4 (&v)[4], uint32_t lane, uint32_t (&d)[16]) {
    const bool b0 = lane & 1u, b1 = lane & 2u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // dword plane k of every chunk
        const uint32_t in[4] = {v[0][k], v[1][k], v[2][k], v[3][k]};
        uint32_t f[4];
        quad_transpose(in, f, b0, b1);
#pragma unroll
        for (int c = 0; c < 4; ++c) d[4 * c + k] = f[c];
    }
}

// Row-swap variant (MODE 4): load_rowswap / rowswap_batch, devutil.hpp.

// Packed frames, the same layout: for instruction j lane 16r + c loads chunk
// r of frame 16j + c (that frame's descriptor fetched from lane 16j + c with
// ds_bpermute), so every instruction consumes whole 64-byte frame lines and
// non-temporal loads pay off; rowswap_batch then gives lane l the first 64
// bytes of its own frame.  (sol `frames_rs_nt` 0.293 ms vs 0.340 ms for one
// frame per lane, C3 IMIX, profiles/r1_frames_rs/.)  Every lane of the wave
// must be active; `ds` is this lane's descriptor (offset << 16 | length; 0
// for lanes past the batch end).  A chunk is read only if it starts inside
// its frame: a 16-byte aligned load that starts at a frame byte stays in
// that byte's page, so nothing past the last frame of the buffer is touched.
// Every lane issues its four loads without a branch: a chunk that starts
// past its frame's end is read from a 16-byte block of zeros instead
// (predicated loads left the compiler's wait counting conservative: an
// s_waitcnt vmcnt(0) that also waited for loads issued after them, such as
// the next batch's descriptors).
__device__ __forceinline__ void load_frames_rs(const uint8_t *__restrict__ frames, uint64_t ds, uint32_t lane,
                                               u32x4 (&v)[4]) {
    const uint32_t lo = static_cast<uint32_t>(ds), hi = static_cast<uint32_t>(ds >> 32);
    const uint32_t chunk = 16u * (lane >> 4);
    const u32x4 *p[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int src = static_cast<int>((16u * j + (lane & 15u)) << 2);
        const uint32_t l = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(lo)));
        const uint32_t h = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(hi)));
        const uint64_t o = (uint64_t(h) << 32 | l) >> 16;
        p[j] = chunk < (l & 0xFFFFu) ? reinterpret_cast<const u32x4 *>(frames + o) + (lane >> 4) : &g_zero16;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load(p[j]);
}

// One lane's frame: the first 64 bytes, chunks past `len` not read (see
// load_frames_rs), then bytes past `len` zeroed.
__device__ __forceinline__ void load16_frame(const uint8_t *__restrict__ p, uint32_t len, uint32_t (&d)[16]) {
    const u32x4 *q = reinterpret_cast<const u32x4 *>(p);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        u32x4 v = u32x4{0, 0, 0, 0};
        if (16u * j < len) v = q[j];
        d[4 * j + 0] = v.x;
        d[4 * j + 1] = v.y;
        d[4 * j + 2] = v.z;
        d[4 * j + 3] = v.w;
    }
    clip16(d, len);
}

// Packet index (within the wave's 64) held by lane l after transpose_batch.
__device__ __forceinline__ uint32_t coal_packet(uint32_t lane) { return 16u * (lane & 3u) + (lane >> 2); }

struct LinearArgs {
    const uint32_t *rec4;
    uint32_t n4;
    const uint32_t *rec6;
    uint32_t n6;
    uint32_t flags;  // NFFACL_PARSE_*
};

// ---------------------------------------------------------------------------
// INDEXED: per-lane interval search + ordered candidate lists (table.hpp).
// ---------------------------------------------------------------------------

struct SlotArgs {
    uint32_t shift, off_dir, off_ent, off_dir16;  // off_dir16: 0 = plain u32 directory
    // flat kernels (generalized slots, table.hpp SlotField): bucket =
    // (key[f1] >> shift) << bits2 | key[f2] >> shift2, key[kFZero] = 0
    uint32_t f1, f2, shift2, bits2;
};
struct FamArgs {
    SlotArgs slot[kMaxSlots];  // INDEXED / LDS forms: [dst addr, src addr, dst port, src port]
    uint32_t off_resid, n_resid;
    uint32_t off_cold;      // HYBRID flat forms: output array (one u32 per rule)
    uint32_t off_ent_base;  // HYBRID flat forms: the family's first entry
};
struct IndexedArgs {
    const uint32_t *tab;    // device table (global memory)
    uint32_t stage_dwords;  // leading dwords staged in LDS (multiple of 4)
    uint32_t flags;         // NFFACL_PARSE_*
    uint32_t dir8;          // HYBRID: two-level directories carry u8 offsets (SplitTab::bounds)
    uint32_t dir16;         // HYBRID: two-level directories (u16 offsets, or u8 with dir8); 0 = plain u32
    uint32_t generic;       // HYBRID flat forms: slots key on SlotArgs::f1/f2 (else slot s on field s)
    uint32_t live;          // positional flat forms: bit s set iff slot s lists rules in some family
    uint32_t off_params;    // flat-LDS positional forms: dword offset (in the LDS image) of the slot
                            // parameter block (table.hpp kFlatParams), 0 = take them from SlotArgs
    FamArgs f4, f6;
    // persistent consumer (service.hip) only: table size for the bounds
    // checks of its global-memory walk, and the host word they flag
    uint32_t tab_dwords;
    uint32_t *oob;
    // batch kernels: batches handed out at run time (engine.hip BatchSource)
    // from the pull heads at `dyn` (nullptr: a fixed grid stride); a pull
    // takes at most dyn_g batches, fewer as a head drains (dyn_wpx: waves
    // per head)
    uint32_t *dyn;
    uint32_t dyn_g, dyn_gmin, dyn_wpx;
};

// Table placement (kernel template argument).
enum TableMode : int {
    kTabGlobal = 0,  // INDEXED, read through L1/L2/MALL
    kTabLds = 1,     // INDEXED, staged whole in LDS
    kTabLdsNP = 9,   // the same for tables that constrain no port
                     // (CompiledTable::ports_any): no L4 port extraction
                     // (no option-port reads) and no port tests
    kTabSplit = 2,   // HYBRID lane form: INDEXED entries in global memory,
                     // directories staged in LDS, one workgroup per CU; the
                     // spare VGPRs buy the frames kernel a two-batch software
                     // pipeline.  (Two workgroups per CU with <= 78 KiB of
                     // directories and 64 VGPRs ran 18 % slower on C3:
                     // longer lists, spills; profiles/r1_hybrid/sw5.)
    kTabFlat = 4,    // HYBRID table, directories read from global memory, the
                     // candidates of a wave's 64 packets tested 64 at a time,
                     // 2 rounds of loads in flight
    kTabFlat4 = 5,   // the same, 4 rounds in flight
    kTabFlatLds = 6, // HYBRID flat-LDS: the flat walk (2 rounds in flight)
                     // over directories staged in LDS, one 1024-thread
                     // workgroup per CU, candidate scratch after the image
    kTabFlatLds4 = 7,  // the same, 4 rounds in flight (larger scratch)
    kTabFlatLds4U = 8, // the same, entry loads of every non-empty round issued
                       // without a per-lane branch (tables with many candidates
                       // per packet: CompiledTable::flat_uncond)
    kTabFlatLdsP = 11, // flat-LDS, positional slots, pipelined walk (classify_flat_pipe,
                       // round 5): family-split candidate streams, one pass's
                       // IPv6 round and IPv4 windows of 4 + 3 rounds in flight together
    kTabFlatLdsG = 10, // flat-LDS over generalized slots (CompiledTable::slots_g:
                       // the coarse / SLOTS2D layout experiments), 4 rounds,
                       // branch-free loads — a kernel of its own, so that the
                       // positional kernels carry no generic lookup code (its
                       // kernel-argument registers spilled in every one of them)
};

extern __shared__ __attribute__((aligned(16))) uint32_t lds_tab[];

// Table accessors: the whole table staged in LDS, or read through L1/L2.
// ld4(i): i is a multiple of 4 (entries are 16-byte aligned, table.hpp), told
// to the compiler so that it emits one ds_read_b128 / global_load_dwordx4 and
// folds the constant part of i into the instruction's offset field (indexing
// in vector units, i >> 2, cost a mask and an add per load: C2's walk -9 %
// VALU instructions).
// List bounds dir[t], dir[t + 1] of a plain u32 directory (one ds_read2 /
// two dword loads).
template <class T>
__device__ __forceinline__ void bounds32(const T &tab, uint32_t dir, uint32_t t, uint32_t &lo, uint32_t &hi) {
    lo = tab.ld(dir + t);
    hi = tab.ld(dir + t + 1);
}

struct LdsTab {
    static constexpr bool kFreeLoads = true;  // out-of-range LDS reads return 0, never fault
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return lds_tab[i]; }
    __device__ __forceinline__ void bounds(uint32_t dir, uint32_t, uint32_t t, uint32_t &lo, uint32_t &hi,
                                           uint32_t = 0) const {
        bounds32(*this, dir, t, lo, hi);
    }
    __device__ __forceinline__ u32x4 ld4(uint32_t i) const {
        __builtin_assume((i & 3u) == 0u);
        return *reinterpret_cast<const u32x4 *>(reinterpret_cast<const char *>(lds_tab) + i * 4u);
    }
};
struct GlobalTab {
    static constexpr bool kFreeLoads = false;
    const uint32_t *__restrict__ p;
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return p[i]; }
    __device__ __forceinline__ void bounds(uint32_t dir, uint32_t, uint32_t t, uint32_t &lo, uint32_t &hi,
                                           uint32_t = 0) const {
        bounds32(*this, dir, t, lo, hi);
    }
    __device__ __forceinline__ u32x4 ld4(uint32_t i) const {
        __builtin_assume((i & 3u) == 0u);
        return *reinterpret_cast<const u32x4 *>(p + i);
    }
};
// List bounds of bucket t from its group's base b and 4-bit counts
// (w1:w0, bucket 16g + i in bits 4i..4i+3): lo = b + the counts before t,
// hi = lo + count(t).  The counts before t are the top 4 (t & 15) bits of
// x << (64 - 4 (t & 15)), summed bytewise (each byte <= 60) by one v_sad_u8.
__device__ __forceinline__ void nib_bounds(uint32_t b, uint32_t w0, uint32_t w1, uint32_t t, uint32_t &lo,
                                           uint32_t &hi) {
    const uint64_t x = uint64_t(w1) << 32 | w0;
    const uint32_t j4 = (t & 15u) * 4u;
    const uint64_t p = (x << (63u - j4)) << 1;  // counts of buckets 0..j-1 in the top bits (j = 0: none)
    const uint32_t pl = static_cast<uint32_t>(p), ph = static_cast<uint32_t>(p >> 32);
    constexpr uint32_t M = 0x0F0F0F0Fu;
    const uint32_t bytes = (pl & M) + ((pl >> 4) & M) + (ph & M) + ((ph >> 4) & M);
    lo = b + __builtin_amdgcn_sad_u8(bytes, 0u, 0u);
    hi = lo + (static_cast<uint32_t>(x >> j4) & 15u);
}

// HYBRID lane form: directories (ld) staged in LDS, entries (ld4) global.
// IN_LDS = false reads the same directory image from global memory (the
// persistent scalar-call consumer, service.hip, which stages nothing).
template <bool IN_LDS>
struct DirTab {
    static constexpr bool kFreeLoads = false;  // entries (ld4) are global
    const uint32_t *__restrict__ p;
    uint32_t limit = 0;  // !IN_LDS: words past the table read as 0 (service.hip)
    __device__ __forceinline__ uint32_t ld(uint32_t i) const {
        if (IN_LDS) return lds_tab[i];
        return i < limit ? p[i] : 0u;
    }
    // two-level directory (table.hpp): dir[t] = base[t >> 6] + dir16[t], or
    // with dir8 (wave-uniform) base[t >> 4] + dir8[t]
    __device__ __forceinline__ void bounds(uint32_t dir, uint32_t dir16, uint32_t t, uint32_t &lo, uint32_t &hi,
                                           uint32_t dir8 = 0) const {
        if (dir16 == 0u) {
            bounds32(*this, dir, t, lo, hi);
            return;
        }
        if (dir8 == 2u) {  // 4-bit counts (table.hpp kDir4GroupShift)
            const uint32_t g = t >> kDir4GroupShift;
            const uint32_t b = ld(dir + g);
            nib_bounds(b, ld(dir16 + 2u * g), ld(dir16 + 2u * g + 1u), t, lo, hi);
            return;
        }
        if (dir8) {
            const uint32_t g = t >> kDir8GroupShift;
            const uint32_t b0 = ld(dir + g), b1 = ld(dir + g + 1);                    // ds_read2
            const uint32_t w0 = ld(dir16 + (t >> 2)), w1 = ld(dir16 + (t >> 2) + 1);  // ds_read2
            const uint32_t x = __builtin_amdgcn_alignbit(w1, w0, (t & 3u) * 8u);  // bytes t, t + 1
            lo = b0 + (x & 0xFFu);
            hi = (((t + 1u) & ((1u << kDir8GroupShift) - 1u)) == 0u ? b1 : b0) + ((x >> 8) & 0xFFu);
            return;
        }
        const uint32_t g = t >> kDir16GroupShift;
        const uint32_t b0 = ld(dir + g), b1 = ld(dir + g + 1);                         // ds_read2
        const uint32_t w0 = ld(dir16 + (t >> 1)), w1 = ld(dir16 + (t >> 1) + 1);      // ds_read2
        const bool odd = (t & 1u) != 0u;
        lo = b0 + (odd ? w0 >> 16 : w0 & 0xFFFFu);
        hi = (((t + 1u) >> kDir16GroupShift) != g ? b1 : b0) + (odd ? w1 & 0xFFFFu : w0 >> 16);
    }
    __device__ __forceinline__ u32x4 ld4(uint32_t i) const {
        __builtin_assume((i & 3u) == 0u);
        return *reinterpret_cast<const u32x4 *>(p + i);
    }
};
using SplitTab = DirTab<true>;

constexpr uint32_t kNone = 0xFFFFFFFFu;

// Per-lane choice between two wave-uniform family parameters (IPv4 / IPv6
// slot arguments).  Both pass through readfirstlane so that they stay in
// SGPRs and the choice is one v_cndmask: written as a plain select of two
// struct fields, the compiler turned it into a select of their ADDRESSES
// and a per-lane global load from the kernel-argument segment — a dependent
// vector-memory round trip per field per batch (C2: 2 per batch, the flat
// C3/C5 kernels: ~25), queued behind the packet stream's loads.
__device__ __forceinline__ uint32_t fam_sel(bool v6, uint32_t x4, uint32_t x6) {
    const uint32_t u4 = __builtin_amdgcn_readfirstlane(x4), u6 = __builtin_amdgcn_readfirstlane(x6);
    return v6 ? u6 : u4;
}

// Mismatch bits of an entry's first 8 dwords (A = words 0..3, B = 4..7):
// address words, protocol (exact flag) and ports — acl.go:526-539 / 546-557
// with IPv6 restricted to the top 32 bits of each address.
template <bool NP = false>
__device__ __forceinline__ uint32_t entry_miss(const u32x4 &A, const u32x4 &B, const Fields &f) {
    const uint32_t proto = ((f.proto ^ B.x) & 0xFFu) & (0u - ((B.x >> 8) & 1u));
    return ((f.s[0] ^ A.x) & A.y) | ((f.t[0] ^ A.z) & A.w) | proto | (NP ? 0u : port_miss(f.ports, B.y, B.z));
}

// Cursor over a table's dwords for the INDEXED walk: LDS tables are walked
// by absolute LDS byte address, which the DS instruction takes as is (a
// dword offset cost a shift and an add of the LDS base per access); other
// tables by dword offset.
typedef __attribute__((address_space(3))) const u32x4 lds_u32x4;
__device__ __forceinline__ uint32_t lds_base() {
    return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const char *)lds_tab));
}
template <class T>
struct Cursor {
    static constexpr bool kLds = std::is_same<T, LdsTab>::value;
    static constexpr uint32_t kScale = kLds ? 4u : 1u;  // cursor units per dword
    __device__ static __forceinline__ uint32_t of(uint32_t i) { return kLds ? lds_base() + 4u * i : i; }
    __device__ static __forceinline__ u32x4 at(const T &tab, uint32_t c, uint32_t dw) {
        if constexpr (kLds) return *(lds_u32x4 *)(uintptr_t)(c + 4u * dw);
        else return tab.ld4(c + dw);
    }
};

// Mismatch bits of the IPv6 extension words 8..19 (address words 1..3) of
// the entry at cursor c.
template <class T>
__device__ __forceinline__ uint32_t entry_miss_ext(const T &tab, uint32_t c, const Fields &f) {
    using C = Cursor<T>;
    const u32x4 x = C::at(tab, c, 8), y = C::at(tab, c, 12), z = C::at(tab, c, 16);
    // x = s1 s2 s3 sm1 | y = sm2 sm3 t1 t2 | z = t3 tm1 tm2 tm3
    return ((f.s[1] ^ x.x) & x.w) | ((f.s[2] ^ x.y) & y.x) | ((f.s[3] ^ x.z) & y.y) |
           ((f.t[1] ^ y.z) & z.y) | ((f.t[2] ^ y.w) & z.z) | ((f.t[3] ^ z.x) & z.w);
}

// Lane mask of a < b (one v_cmp into an SGPR pair).  A ballot of a combined
// condition compiled to v_cndmask + v_cmp first: two VALU per ballot.
__device__ __forceinline__ uint64_t lanes_lt(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_uicmp(a, b, 36 /* ICMP_ULT */);
}

// x * entry dwords (IPv6 20, IPv4 8): one full-rate 24-bit multiply (entry
// numbers < 2^24).  (Written as two shift forms under a select, it compiled
// to a divergent branch per slot with a quarter-rate v_mul_lo_u32 in it.)
__device__ __forceinline__ uint32_t times_ew(uint32_t x, bool v6) { return __umul24(x, v6 ? 20u : 8u); }

// First match over the four key slots of the lane's family, walked together:
// every iteration tests the next entry of every slot list, so the wave pays
// max(list lengths) table round trips, not their sum.  Loops run while some
// lane has work (lane masks from v_cmp, no ballot of combined conditions);
// the IPv6 extension words are read under a plain per-lane branch.
// U = list entries per slot per loop trip: all NS x U entry loads of a trip
// are issued before any is tested.  The walk keeps cursors (Cursor<T>) per
// slot, advanced by adds.  Tables whose reads are free to issue for every
// lane (T::kFreeLoads: LDS, where an inactive lane's read is harmless and
// cheaper than the exec-mask juggling and register zeroing a predicated load
// needs) load unconditionally; global tables load only for lanes still
// walking (a 16-byte load costs the TA 16 cycles per 64 active lanes; global:
// -4 % on C3, profiles/r1_masked).  LDS tables (offsets < 2^16 dwords) get
// their per-family slot parameters as 16-bit halves of one SGPR each, one
// v_bfe per parameter instead of two moves and a select.
// LDS walks, done lanes (NFFACL_EXP_LDSDEAD, an experiment build option):
// 0 (default) a done lane's cursor stays at its list end and its
// unconditional entry reads hit a random entry; 1 its cursor moves past the
// LDS allocation (kDeadCursor > every list end, so the loop test stays one
// v_cmp) and its reads return 0 without touching a bank; 2 predicated reads.
// On C2, 1 cuts LDS bank-conflict cycles from 35 M to 11 M per launch but
// runs 3.5 % slower (0.2235-0.2260 vs 0.2156-0.2163 ms; 2: 0.2235-0.2239),
// profiles/r4_ab/lds_dead/: the conflicts cost LDS cycles the kernel has to
// spare, the extra select costs issue slots it has not.
#ifndef NFFACL_EXP_LDSDEAD
#define NFFACL_EXP_LDSDEAD 0
#endif
constexpr uint32_t kDeadCursor = 0xFFFF0000u;

template <int NS, int U, class T, bool NP = false>
__device__ __forceinline__ uint32_t classify_indexed(const T &tab, const IndexedArgs &a, const Fields &f) {
    using C = Cursor<T>;
    constexpr bool kDead = C::kLds && NFFACL_EXP_LDSDEAD == 1;
    constexpr bool kPred = C::kLds && NFFACL_EXP_LDSDEAD == 2;
    const bool v6 = f.is6;
    const bool mine = f.is4 || f.is6;
    const uint32_t ew = v6 ? kEnt6Dwords : kEnt4Dwords;
    const uint32_t key[4] = {__builtin_bswap32(f.t[0]), __builtin_bswap32(f.s[0]), f.ports >> 16,
                             f.ports & 0xFFFFu};
    const uint32_t half = v6 ? 16u : 0u;
    auto par = [&](uint32_t x4, uint32_t x6) -> uint32_t {
        if constexpr (C::kLds) return __builtin_amdgcn_ubfe(__builtin_amdgcn_readfirstlane(x4 | x6 << 16), half, 16);
        else return fam_sel(v6, x4, x6);
    };
    uint32_t c[NS], e[NS];  // cursors: the slot list's next entry, its end
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const SlotArgs &s4 = a.f4.slot[s], &s6 = a.f6.slot[s];
        const uint32_t shift = par(s4.shift, s6.shift);
        const uint32_t dir = par(s4.off_dir, s6.off_dir);
        const uint32_t base = par(s4.off_ent, s6.off_ent);
        const uint32_t t = key[s] >> shift;  // < n_buckets for any key: both reads in range
        uint32_t lo, hi;
        tab.bounds(dir, C::kLds ? 0u : fam_sel(v6, s4.off_dir16, s6.off_dir16), t, lo, hi, a.dir8);
        c[s] = C::of(base + times_ew(lo, v6));
        // (a select of the bound, not of the cursor: otherwise the compiler
        // sank the hi read into a branch, two LDS round trips instead of one)
        e[s] = C::of(base + times_ew(mine ? hi : lo, v6));
        if (kDead) c[s] = c[s] < e[s] ? c[s] : kDeadCursor;
    }
    const uint32_t cstep = C::kScale * ew;  // one entry in cursor units
    uint32_t best = kNone, out = 0;
    while (true) {
        uint64_t any = 0;
#pragma unroll
        for (int s = 0; s < NS; ++s) any |= lanes_lt(c[s], e[s]);
        if (any == 0u) break;
        u32x4 A[NS][U], B[NS][U];
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t cu = c[s] + u * cstep;
                if (T::kFreeLoads && !kPred) {
                    A[s][u] = C::at(tab, cu, 0);
                    B[s][u] = C::at(tab, cu, 4);
                } else {
                    A[s][u] = B[s][u] = u32x4{0, 0, 0, 0};
                    if (cu < e[s]) {
                        A[s][u] = C::at(tab, cu, 0);
                        B[s][u] = C::at(tab, cu, 4);
                    }
                }
            }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            bool go = true;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t cu = c[s] + u * cstep;
                const bool act = go && cu < e[s];
                const uint32_t idx = B[s][u].x >> kEntIndexShift;
                const bool earlier = act && idx < best;
                bool pass = entry_miss<NP>(A[s][u], B[s][u], f) == 0u;
                if (v6 && earlier && pass) pass = entry_miss_ext(tab, cu, f) == 0u;
                const bool take = earlier && pass;
                best = take ? idx : best;
                out = take ? B[s][u].w : out;
                // stop at a hit, or once the ascending list has passed `best`
                go = earlier && !pass;
            }
            c[s] = go ? c[s] + U * cstep : (kDead ? kDeadCursor : e[s]);
        }
    }
    // rules with no selective key: wave-uniform scan in rule order per family
#pragma unroll
    for (int fam = 0; fam < 2; ++fam) {
        const FamArgs &fa = fam ? a.f6 : a.f4;
        const bool in_fam = fam ? f.is6 : f.is4;
        const uint32_t w = fam ? kEnt6Dwords : kEnt4Dwords;
        if (fa.n_resid == 0u) continue;
        const uint64_t fam_lanes = ballot(in_fam);
        for (uint32_t i = 0; i < fa.n_resid; ++i) {
            const uint32_t cu = C::of(fa.off_resid + i * w);
            const u32x4 A = C::at(tab, cu, 0), B = C::at(tab, cu, 4);
            const uint32_t idx = B.x >> kEntIndexShift;
            if ((lanes_lt(idx, best) & fam_lanes) == 0u) break;  // residual list ascends too
            bool pass = in_fam && idx < best && entry_miss<NP>(A, B, f) == 0u;
            if (fam && pass) pass = entry_miss_ext(tab, cu, f) == 0u;
            best = pass ? idx : best;
            out = pass ? B.w : out;
        }
    }
    return best != kNone ? out : 0u;
}

// The leading stage_dwords of the table into LDS, once per workgroup.  Each
// thread issues up to U 16-byte loads before its first LDS write (a plain
// copy loop waited out one HBM round trip per 16 KiB: 4-7 in a row at the
// start of every C2/C3/C5 launch).
__device__ __forceinline__ void stage_table(const IndexedArgs &a) {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a.tab);
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds_tab);
    const uint32_t nv = a.stage_dwords / 4, step = blockDim.x;
    constexpr uint32_t U = 8;
    for (uint32_t i0 = threadIdx.x; i0 < nv; i0 += U * step) {
        u32x4 v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
            if (i0 + u * step < nv) v[u] = src[i0 + u * step];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
            if (i0 + u * step < nv) dst[i0 + u * step] = v[u];
    }
    __syncthreads();
}

// ---- HYBRID (table.hpp "hybrid table") --------------------------------------

// 12-byte pieces of the exact flat-form entries (table.hpp): an IPv4 entry
// is two (the compiler issues dwordx4 + dwordx2), an IPv6 entry four.
typedef uint32_t u32x3 __attribute__((ext_vector_type(3), aligned(4)));

__device__ __forceinline__ u32x3 ld3(const uint32_t *__restrict__ p) { return *reinterpret_cast<const u32x3 *>(p); }

// Pair gathers (round 6): the two lanes of a pair (2i, 2i + 1) read ONE
// candidate's entry per load instruction — the even lane a 12-byte piece, the
// odd lane the next — so a wave instruction touches 32 entries' lines, not 64.
// Scattered loads cost the TA/TCP a cycle per line touched (prof_r6_c5: TA
// busy 85 % of the kernel's cycles, VALU 17 %, LDS 13 %).  The pair's loads:
// X = the even lane's candidate's pieces (p | p + 1), Y = the odd lane's; then
// pair_unpack trades across the pair (one DPP move per word, unconditional,
// both arms of the selects) so that every lane holds its own candidate's
// pieces p in X and p + 1 in Y — what two plain loads would have given it.
// Measured (profiles/r6_ab/pair/): C5 0.5084 / 0.5058 and 0.5136 / 0.5224 ms
// vs 0.5246 / 0.5235 and 0.5275 / 0.5241 without — 1.5-3 %, not the halving a
// per-line TA cost predicts: the L2 requests (one per entry line, unchanged)
// and their latency set the rest.  In classify_flat (C3) the same loads ran
// even (0.408 / 0.409 vs 0.413 / 0.407 ms) and were not kept; the pipelined
// walk uses them.
#ifndef NFFACL_PAIR_GATHER
#define NFFACL_PAIR_GATHER 1
#endif
__device__ __forceinline__ void pair_offsets(uint32_t o, bool odd, uint32_t &oe, uint32_t &od) {
    const uint32_t p = dpp<0xB1>(o);  // quad_perm [1,0,3,2]: the partner's offset
    oe = (odd ? p : o) + (odd ? 12u : 0u);
    od = (odd ? o : p) + (odd ? 12u : 0u);
}
__device__ __forceinline__ void pair_unpack(bool odd, u32x3 &X, u32x3 &Y) {
    u32x3 lo, hi;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const uint32_t r = dpp<0xB1>(odd ? X[c] : Y[c]);
        lo[c] = odd ? r : X[c];
        hi[c] = odd ? Y[c] : r;
    }
    X = lo;
    Y = hi;
}

// Position of the first set bit from the top (v_ffbh_u32), 0xFFFFFFFF for 0
// — defined here for 0, unlike __builtin_clz (hence the one-line asm).
__device__ __forceinline__ uint32_t ffbh_raw(uint32_t x) {
    uint32_t r;
    asm("v_ffbh_u32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// Does an exact entry's first six words (both families) reject the packet?
// Top address words under their prefix lengths (IPv6: the top word, any
// length), protocol, ports — acl.go:526-539 / 546-557 for IPv4 completely,
// for IPv6 up to the low address words.  ks/kd: big-endian src/dst (top)
// words.  An address word x = key ^ rule misses its prefix of length L iff
// its first differing bit lies above L: ffbh(x) < L (x = 0: 0xFFFFFFFF, no
// miss at any L; L >= 32 with x != 0: a miss), one compare, no mask.
// (Round 6: the masks were 0xFFFFFFFF00000000 >> L, one v_lshrrev_b64 each;
// a 64-bit instruction whose 32-bit operand is the allocation's last VGPR
// reads the next wave's v0 on MI355X — the NS = 7 pipelined walk's wrong
// verdicts, DESIGN.md §4.3 — so no kernel shifts by a variable 64 bits here.)
__device__ __forceinline__ bool hyb_miss(const u32x3 &A, const u32x3 &B, uint32_t ks, uint32_t kd, uint32_t proto,
                                         uint32_t ports) {
    const uint32_t sl = B.z & 0xFFu, dl = (B.z >> 8) & 0xFFu;
    const uint32_t pm = ((proto ^ A.z) & 0xFFu) & (0u - ((A.z >> 8) & 1u));
    const bool ms = ffbh_raw(ks ^ A.x) < sl, md = ffbh_raw(kd ^ A.y) < dl;
    return ms || md || (pm | port_miss(ports, B.x, B.y)) != 0u;
}

// IPv6 address words 1..3 of an exact entry (C = src1 src2 src3, D = dst1
// dst2 dst3) against big-endian packet words s[1..3], t[1..3].
// By first difference: the address matches its prefix of length L iff its
// first bit differing from the rule's (counted from bit 32) lies at or past
// L - 32 (v_ffbh per word instead of three prefix masks per address).
__device__ __forceinline__ uint32_t first_diff96(uint32_t x1, uint32_t x2, uint32_t x3) {
    const uint32_t p1 = __clz(x1), p2 = 32u + __clz(x2), p3 = 64u + __clz(x3);  // __clz(0) = 32
    return x1 != 0u ? p1 : x2 != 0u ? p2 : p3;
}

__device__ __forceinline__ bool hyb_miss6(const u32x3 &C, const u32x3 &D, uint32_t lens, const uint32_t (&s)[4],
                                          const uint32_t (&t)[4]) {
    const uint32_t sl = lens & 0xFFu, dl = (lens >> 8) & 0xFFu;
    const uint32_t ps = 32u + first_diff96(s[1] ^ C.x, s[2] ^ C.y, s[3] ^ C.z);
    const uint32_t pd = 32u + first_diff96(t[1] ^ D.x, t[2] ^ D.y, t[3] ^ D.z);
    return ps < sl || pd < dl;
}

// ---- FLAT: a wave's candidates, 64 at a time --------------------------------
//
// The list walks above cost one dependent table round trip per loop trip, and
// a wave takes as many trips as its longest walk.  For tables that live in
// L2/MALL that latency, not bandwidth, bounds the kernel (C5: 13 trips of
// ~3 us per 64 packets).  Here every lane first looks up the list bounds of
// its packet in each slot (one round trip), the wave lays all (packet, slot,
// entry) candidates end to end (exclusive scan of the list lengths), and
// round r gives lane l candidate 64 r + l: one table load per lane per round,
// all 64 lanes busy, ceil(total / 64) rounds.  A lane finds its candidate's
// list through an LDS window: every list overlapping the round's 64
// positions marks its first position there, a prefix max over the window
// carries the mark forward.  Each passing candidate posts its rule index to
// the packet's LDS minimum (ds_min_u32): the minimum over every candidate is
// the first match of the ordered lists, no early exit needed.
template <int R>
struct FlatScratch {
    // window position -> (owner lane << 19 | slot << 16 | position << 8 | owner's protocol) + 1, 0 = none
    // (ascending with the position, as the prefix max needs; the protocol
    // rides along so that the owner's fields take three ds_bpermute, not four)
    uint32_t mark[64 * R];
    uint32_t delta[64 * R];  // window position -> (entry number - candidate number) << 1 | IPv6
    uint64_t best[64];       // per packet (lane): lowest passing rule index << 32 | output code
};

// Complete the load that produced `x` here, inside the (rare) branch that
// issued it.  Left pending across the join, it made the compiler wait for
// every outstanding vector-memory operation at the value's next use — the
// batch's own verdict stores included, one HBM write round trip per batch.
__device__ __forceinline__ void settle(uint32_t &x) { asm volatile("" : "+v"(x)); }

// Order this wave's LDS writes before its following LDS reads of other lanes'
// words (one wave: program order on the LDS queue; this keeps the compiler
// from reordering across it).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t src_lane) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(src_lane << 2), static_cast<int>(v)));
}

// Wave-wide inclusive scans on DPP (GFX9 controls): row_shr 1, 2, 4, 8 build
// the prefix inside each 16-lane row, row_bcast:15 (rows 1, 3) and
// row_bcast:31 (rows 2, 3) carry the row totals.  Lanes without a source read
// 0 (bound_ctrl), the identity of both + and max over unsigned values.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), CTRL, ROW_MASK, 0xF, true));
}

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
    x += dpp0<0x111>(x);
    x += dpp0<0x112>(x);
    x += dpp0<0x114>(x);
    x += dpp0<0x118>(x);
    x += dpp0<0x142, 0xA>(x);
    x += dpp0<0x143, 0xC>(x);
    return x;
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = max(x, dpp0<0x111>(x));
    x = max(x, dpp0<0x112>(x));
    x = max(x, dpp0<0x114>(x));
    x = max(x, dpp0<0x118>(x));
    x = max(x, dpp0<0x142, 0xA>(x));
    x = max(x, dpp0<0x143, 0xC>(x));
    return x;
}

template <int NS, int R, bool LDS_DIRS, bool UNCOND = false, bool DIRS_IN_LDS = true, bool GEN = false>
__device__ __forceinline__ uint32_t classify_flat(const IndexedArgs &a, const Fields &f, FlatScratch<R> &W,
                                                  uint32_t lane) {
    const bool v6 = f.is6;
    const bool mine = f.is4 || f.is6;
    // The persistent consumer (DIRS_IN_LDS == false) reads the table with
    // bounds checks: a word outside it reads as 0 and raises the host flag
    // a.oob (reported by nffacl_service_get_stats) instead of faulting.
    auto g3 = [&](const uint32_t *p) -> u32x3 {
        if (!DIRS_IN_LDS) {
            const uint64_t off = static_cast<uint64_t>(p - a.tab);
            if (off + 3u > a.tab_dwords) {
                __hip_atomic_store(a.oob, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                return u32x3{0, 0, 0};
            }
        }
        return ld3(p);
    };
    auto g1 = [&](uint32_t i) -> uint32_t {
        if (!DIRS_IN_LDS && i >= a.tab_dwords) {
            __hip_atomic_store(a.oob, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return 0u;
        }
        return a.tab[i];
    };
    const uint32_t ks = __builtin_bswap32(f.s[0]), kd = __builtin_bswap32(f.t[0]);
    const uint32_t sport = f.ports & 0xFFFFu, dport = f.ports >> 16;
    // key[f] of a slot field f (SlotField; kFZero and unused slots: 0)
    auto pick = [&](uint32_t fld) -> uint32_t {
        return fld == kFDst ? kd : fld == kFSrc ? ks : fld == kFDport ? dport : fld == kFSport ? sport : 0u;
    };
    // list bounds of this packet in every slot (family-relative entry numbers)
    uint32_t st[NS], ln[NS];
    // positional slots (a.generic == 0: slot s keys on field s, 1-D): the key
    // is known at compile time, no per-lane field selects (wave-uniform branch)
    if (LDS_DIRS && !GEN) {
        // directories staged in LDS: offsets < 2^16 dwords, so the family
        // parameters travel as 16-bit SGPR halves (one v_bfe each, as in
        // classify_indexed); global directories (service.hip): fam_sel
        const uint32_t half = v6 ? 16u : 0u;
        auto par = [&](uint32_t x4, uint32_t x6) -> uint32_t {
            if (DIRS_IN_LDS) return __builtin_amdgcn_ubfe(__builtin_amdgcn_readfirstlane(x4 | x6 << 16), half, 16);
            return fam_sel(v6, x4, x6);
        };
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const SlotArgs &s4 = a.f4.slot[s], &s6 = a.f6.slot[s];
            if (!((a.live >> s) & 1u)) {  // empty in both families (wave-uniform): no lookup
                st[s] = 0u;
                ln[s] = 0u;
                continue;
            }
            // the slot's parameters: one broadcast ds_read_b128 of the
            // table's LDS parameter block (kFlatParams; every flat-LDS
            // positional table has one) — kept as kernel arguments they held
            // 2 SGPRs per slot and family across the batch loop and spilled
            // (C5 NS = 6: 113 SGPR spills, 320 v_readlane in the loop); the
            // service's walk (directories in global memory) takes SlotArgs
            uint32_t shift, dir, dir16, bits2 = 0, shift2 = 0;
            if (DIRS_IN_LDS) {
                const u32x4 P = *(lds_u32x4 *)(uintptr_t)(lds_base() + 4u * (a.off_params + kFlatParamDwords * s));
                shift = __builtin_amdgcn_ubfe(P.x, half, 16);
                dir = __builtin_amdgcn_ubfe(P.y, half, 16);
                dir16 = __builtin_amdgcn_ubfe(P.z, half, 16);
                const uint32_t fine = __builtin_amdgcn_ubfe(P.w, half, 16);
                bits2 = fine & 0xFFu;
                shift2 = fine >> 8;
            } else {
                shift = par(s4.shift, s6.shift);
                dir = par(s4.off_dir, s6.off_dir);
                dir16 = par(s4.off_dir16, s6.off_dir16);
                if (s >= 4) {
                    bits2 = par(s4.bits2, s6.bits2);
                    shift2 = par(s4.shift2, s6.shift2);
                }
            }
            uint32_t t;
            if (s < 4) {  // 1-D: [dst, src, dport, sport]
                const uint32_t key = s == kFDst ? kd : s == kFSrc ? ks : s == kFDport ? dport : sport;
                t = key >> shift;
            } else {      // fine 2-D grids: [dst x dport, src x dport, dst x sport, src x sport]
                const uint32_t addr = (s & 1) ? ks : kd, port = s < 6 ? dport : sport;
                t = ((addr >> shift) << bits2) | (port >> shift2);
            }
            uint32_t hi;
            DirTab<DIRS_IN_LDS>{a.tab, a.tab_dwords}.bounds(dir, dir16, t, st[s], hi, a.dir8);
            ln[s] = mine ? hi - st[s] : 0u;
        }
    } else {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const SlotArgs &s4 = a.f4.slot[s], &s6 = a.f6.slot[s];
        const uint32_t shift = fam_sel(v6, s4.shift, s6.shift);
        const uint32_t dir = fam_sel(v6, s4.off_dir, s6.off_dir);
        const uint32_t t = ((pick(fam_sel(v6, s4.f1, s6.f1)) >> shift) << (fam_sel(v6, s4.bits2, s6.bits2))) |
                           (pick(fam_sel(v6, s4.f2, s6.f2)) >> (fam_sel(v6, s4.shift2, s6.shift2)));
        if (LDS_DIRS) {
            uint32_t hi;
            DirTab<DIRS_IN_LDS>{a.tab, a.tab_dwords}.bounds(dir, fam_sel(v6, s4.off_dir16, s6.off_dir16), t, st[s], hi, a.dir8);
            ln[s] = mine ? hi - st[s] : 0u;
        } else {
            // generalized slots: a family's unused slots (f1 == kFZero) read nothing
            st[s] = 0u;
            ln[s] = 0u;
            if (mine && (fam_sel(v6, s4.f1, s6.f1)) != kFZero) {
                st[s] = g1(dir + t);
                ln[s] = g1(dir + t + 1) - st[s];
            }
        }
    }
    }
    uint32_t total = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) total += ln[s];
    const uint32_t incl = wave_incl_sum(total);
    const uint32_t off = incl - total;  // first candidate number of this packet
    const uint32_t T = __builtin_amdgcn_readlane(incl, 63);
    W.best[lane] = ~0ull;
    const uint32_t *__restrict__ E4 = a.tab + a.f4.off_ent_base;
    const uint32_t *__restrict__ E6 = a.tab + a.f6.off_ent_base;
    // One window of RR rounds (64 RR candidates) starting at candidate `win`,
    // straight-line so the compiler interleaves its RR rounds of loads.  A
    // window of R rounds runs while at least 64 (R - 1) + 1 candidates
    // remain; the last window runs only the rounds its candidates fill (one
    // wave-uniform dispatch on the remainder, not a branch per round: per-round
    // branches broke the load interleave, profiles/r2_exact/skip/).
    auto window = [&](uint32_t win, auto rr) {
        constexpr int RR = decltype(rr)::value;
#pragma unroll
        for (int j = 0; j < RR; ++j) W.mark[64 * j + lane] = 0u;
        wave_lds_sync();
        uint32_t so = off;  // candidate number of list s's first entry
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (ln[s] != 0u && so < win + 64u * RR && so + ln[s] > win) {
                const uint32_t pos = so > win ? so - win : 0u;
                W.mark[pos] = (lane << 19 | static_cast<uint32_t>(s) << 16 | pos << 8 | (f.proto & 0xFFu)) + 1u;
                if (DIRS_IN_LDS) {
                    // byte offset (from a.tab) of the list's "candidate 0"
                    // entry, wrapping mod 2^32, IPv6 in bit 0: the round's
                    // entry address is then one multiply-shift-add away
                    const uint32_t w = v6 ? kHybEnt6Dwords : kHybEnt4Dwords;
                    const uint32_t fb = v6 ? a.f6.off_ent_base : a.f4.off_ent_base;
                    // (signed 24-bit multiply, full rate: |st - so| < 2^23,
                    // table_consistent; a 32-bit v_mul_lo_u32 is quarter rate)
                    W.delta[pos] = ((fb + static_cast<uint32_t>(__mul24(static_cast<int>(st[s] - so), static_cast<int>(w))))
                                    << 2) | (v6 ? 1u : 0u);
                } else {
                    W.delta[pos] = ((st[s] - so) << 1) | (v6 ? 1u : 0u);
                }
            }
            so += ln[s];
        }
        wave_lds_sync();
        // RR rounds: locate every candidate's list, then issue every round's
        // entry loads (IPv6 candidates: all four pieces) before testing any.
        // Rounds 0..RR-2 are full (the dispatch below), only round RR-1 can
        // hold lanes past the wave's candidates (the per-round k < T test
        // stays: with it compiled out the scheduler hoists more loads, and
        // the frames kernels spill at 128 VGPRs).
        uint32_t owner[RR], idx[RR], oproto[RR];
        bool valid[RR], six[RR];
        u32x3 A[RR], B[RR], C[RR], D[RR];
        // the rounds' prefix-max scans are independent (only their carries
        // chain): issued together, their DPP steps interleave instead of
        // waiting out each other's data hazards
        uint32_t scan[RR];
#pragma unroll
        for (int j = 0; j < RR; ++j) scan[j] = wave_incl_max(W.mark[64 * j + lane]);
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            const uint32_t m = max(scan[j], carry);
            if (j + 1 < RR) carry = __builtin_amdgcn_readlane(m, 63);
            const uint32_t k = win + 64u * j + lane;
            valid[j] = k < T;
            owner[j] = (m - 1u) >> 19;
            oproto[j] = (m - 1u) & 0xFFu;
            const uint32_t dp = W.delta[((m - 1u) >> 8) & 0xFFu];
            six[j] = (dp & 1u) != 0u;
            // UNCOND: lanes past the wave's candidates load entry 0 of the
            // IPv4 list (untested) instead of branching around the load
            // (profiles/r2_exact/uncond/).  (Round 3: window-relative entry
            // offsets with one 24-bit multiply-add per candidate — fewer VALU
            // per round, more per window and +7-11 VGPRs — ran C3 0.502 vs
            // 0.472 ms, C5 even; profiles/r3_ab/)
            const uint32_t ent = !UNCOND || valid[j] ? k + static_cast<uint32_t>(static_cast<int32_t>(dp) >> 1) : 0u;
            // (entry numbers < 2^24, table_consistent: a full-rate 24-bit multiply)
            const bool e6 = six[j] && (!UNCOND || valid[j]);
            // (round 4: one uniform base + a 32-bit byte offset per entry, the
            // saddr load form, -56 static VALU: C5 0.6547 / 0.6527 vs 0.6520 /
            // 0.6491 ms, C3 even; profiles/r4_ab/saddr/ — not kept)
            // staged walks: entry byte offset = delta + k * 24 (IPv4) / 48
            // (IPv6), no family base select (round 4: C5 0.5915 / 0.5936 vs
            // 0.6004 / 0.5984 ms, C3 0.4001 / 0.4058 vs 0.4084 / 0.4053;
            // profiles/r4_ab/bdelta/); the consumer's walk keeps entry numbers
            const uint32_t *e;
            if (DIRS_IN_LDS) {
                const uint32_t off = !UNCOND || valid[j] ? (dp & ~3u) + (__umul24(k, 4u * kHybEnt4Dwords) << (dp & 1u))
                                                         : (a.f4.off_ent_base << 2);
                e = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(a.tab) + off);
            } else {
                e = (e6 ? E6 : E4) + __umul24(ent, e6 ? kHybEnt6Dwords : kHybEnt4Dwords);
            }
            if (UNCOND || valid[j]) {
                A[j] = g3(e);
                B[j] = g3(e + 3);
            } else {
                A[j] = B[j] = u32x3{0, 0, 0};
            }
            if (valid[j] && six[j]) {  // (C, D are read only for valid IPv6 candidates)
                C[j] = g3(e + 6);
                D[j] = g3(e + 9);
            }
        }
        bool pass[RR];
        bool any6 = false;
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            // the owner packet's fields
            const uint32_t o = owner[j];
            const uint32_t oks = bperm(ks, o), okd = bperm(kd, o);
            const uint32_t opt = bperm(f.ports, o);
            pass[j] = valid[j] && !hyb_miss(A[j], B[j], oks, okd, oproto[j], opt);
            idx[j] = A[j].z >> kEntIndexShift;
            any6 |= pass[j] && six[j];
        }
        if (ballot(any6)) {  // IPv6 candidates: address words 1..3 of the owner
            uint32_t sb[4], tb[4];
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                sb[q] = __builtin_bswap32(f.s[q]);
                tb[q] = __builtin_bswap32(f.t[q]);
            }
#pragma unroll
            for (int j = 0; j < RR; ++j) {
                if (ballot(pass[j] && six[j])) {  // whole wave: bpermute reads every lane
                    uint32_t os[4] = {0, 0, 0, 0}, ot[4] = {0, 0, 0, 0};
#pragma unroll
                    for (int q = 1; q < 4; ++q) {
                        os[q] = bperm(sb[q], owner[j]);
                        ot[q] = bperm(tb[q], owner[j]);
                    }
                    if (pass[j] && six[j]) pass[j] = !hyb_miss6(C[j], D[j], B[j].z, os, ot);
                }
            }
        }
        // (posting from every lane, ~0 to its own word when nothing passed,
        // instead of the branch: C5 0.757 vs 0.750 ms, profiles/r2_exact/uncond/am_*)
#pragma unroll
        for (int j = 0; j < RR; ++j)  // rule index << 32 | output code: the minimum carries the winner's output
            if (pass[j]) atomicMin(reinterpret_cast<unsigned long long *>(&W.best[owner[j]]),
                                   static_cast<unsigned long long>(idx[j]) << 32 | (B[j].z >> kHybOutShift));
        wave_lds_sync();
    };
    // (a mark carries its window position in 8 bits: at most 256 positions,
    // R <= 4 — an R = 5 experiment build faulted the GPU on out-of-range
    // entry numbers in round 4)
    static_assert(R >= 1 && R <= 4, "window positions are 8-bit fields of the marks");
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, (R >= 3 ? 3 : R)>;
    using IR = std::integral_constant<int, R>;
    for (uint32_t win = 0; win < T; win += 64 * R) {
        const uint32_t rem = T - win;  // wave-uniform
        if (rem > 64u * (R - 1)) window(win, IR{});
        else if (R >= 3 && rem > 128u) window(win, I3{});
        else if (rem > 64u) window(win, I2{});
        else window(win, I1{});
    }
    uint64_t best = W.best[lane];  // ~0 or rule index << 32 | output code
    // rules with no selective key: wave-uniform scan in rule order per family
#pragma unroll
    for (int fam = 0; fam < 2; ++fam) {
        const FamArgs &fa = fam ? a.f6 : a.f4;
        const bool in_fam = fam ? f.is6 : f.is4;
        const uint32_t ew = fam ? kHybEnt6Dwords : kHybEnt4Dwords;
        for (uint32_t i = 0; i < fa.n_resid; ++i) {
            const uint32_t *e = a.tab + fa.off_resid + i * ew;
            const u32x3 RA = g3(e), RB = g3(e + 3);
            const uint32_t ri = RA.z >> kEntIndexShift;
            const bool want = in_fam && ri < uint32_t(best >> 32);
            if (!ballot(want)) break;  // residual list ascends too
            bool ok = want && !hyb_miss(RA, RB, ks, kd, f.proto, f.ports);
            if (fam && ballot(ok)) {
                uint32_t sb[4] = {0, 0, 0, 0}, tb[4] = {0, 0, 0, 0};
#pragma unroll
                for (int q = 1; q < 4; ++q) {
                    sb[q] = __builtin_bswap32(f.s[q]);
                    tb[q] = __builtin_bswap32(f.t[q]);
                }
                if (ok) ok = !hyb_miss6(g3(e + 6), g3(e + 9), RB.z, sb, tb);
            }
            best = ok ? (uint64_t(ri) << 32 | (RB.z >> kHybOutShift)) : best;
        }
    }
    // output numbers below kHybOutEscape travel in the entry; others come from the output array
    const bool hit = best != ~0ull;
    uint32_t out = hit ? static_cast<uint32_t>(best) : 0u;
    const bool rd = hit && out == kHybOutEscape;
    if (ballot(rd)) {
        const uint32_t r = static_cast<uint32_t>(best >> 32);
        if (rd) out = g1(fam_sel(v6, a.f4.off_cold, a.f6.off_cold) + r);
        settle(out);
    }
    return out;
}

// ---- FLAT, pipelined (round 5): family-split windows, a batch's rounds in flight together ----
//
// classify_flat (above) runs a batch's candidates window by window: marks,
// scans, entry loads of 4 rounds, then their tests, and only then the next
// window — C5 (6.5 candidates per packet, 7 rounds) waits out two dependent
// entry round trips per batch, and every round carries the IPv6 machinery
// (12-dword entries, a per-round ballot and stage for address words 1..3)
// although IPv6 candidates are ~7 % of the total.  Here:
//  * the candidates are laid out per family: the IPv4 packets' lists form one
//    stream, the IPv6 packets' another, each with its own exclusive scan;
//  * a pass marks, locates and issues the loads of up to one IPv6 round and
//    IPv4 windows of 4 and 3 rounds — the window scratch (marks, deltas) is
//    free again once a window's candidates are located, so the LDS footprint
//    is classify_flat's — and tests them only once the loads behind them are
//    in flight (IPv6 round and first window issued, IPv6 round tested, second
//    window issued, both windows tested): about one exposed entry round trip
//    per batch (C5: 390 IPv4 + 27 IPv6 candidates per batch, one pass);
//  * IPv4 rounds hold 6-dword entries and test them with no IPv6 branch; the
//    IPv6 round tests all of its lanes' address words 1..3 at once;
//  * directory lookups are straight-line over every slot (the form is a
//    wave-uniform table property), so their LDS reads overlap.
// Semantics are classify_flat's: the minimum (rule index << 32 | output code)
// over all candidates that pass the full rule test is the first match
// (acl.go:522-565), residual entries after.  Positional slots, directories
// and parameter block staged in LDS (flat-LDS tables).

// List bounds of this packet in every positional slot (directories in LDS).
template <int NS>
__device__ __forceinline__ void flat_bounds_lds(const IndexedArgs &a, const Fields &f, uint32_t (&st)[NS],
                                                uint32_t (&ln)[NS]) {
    const bool v6 = f.is6;
    const bool mine = f.is4 || f.is6;
    const uint32_t ks = __builtin_bswap32(f.s[0]), kd = __builtin_bswap32(f.t[0]);
    const uint32_t sport = f.ports & 0xFFFFu, dport = f.ports >> 16;
    const uint32_t half = v6 ? 16u : 0u;
    // every slot's parameters first (broadcast ds_read_b128 each), then the
    // bucket reads: no slot waits for another's LDS round trip
    u32x4 P[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s)
        P[s] = *(lds_u32x4 *)(uintptr_t)(lds_base() + 4u * (a.off_params + kFlatParamDwords * s));
    uint32_t t[NS], dir[NS], d16[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const uint32_t shift = __builtin_amdgcn_ubfe(P[s].x, half, 16);
        dir[s] = __builtin_amdgcn_ubfe(P[s].y, half, 16);
        d16[s] = __builtin_amdgcn_ubfe(P[s].z, half, 16);
        if (s < 4) {  // 1-D: [dst, src, dport, sport]
            const uint32_t key = s == kFDst ? kd : s == kFSrc ? ks : s == kFDport ? dport : sport;
            t[s] = key >> shift;
        } else {      // fine 2-D grids: [dst x dport, src x dport, dst x sport, src x sport]
            const uint32_t fine = __builtin_amdgcn_ubfe(P[s].w, half, 16);
            const uint32_t addr = (s & 1) ? ks : kd, port = s < 6 ? dport : sport;
            t[s] = ((addr >> shift) << (fine & 0xFFu)) | (port >> (fine >> 8));
        }
    }
    auto lds2 = [](uint32_t dw, uint32_t &x, uint32_t &y) {  // one ds_read2_b32 (or b64 when aligned)
        x = lds_tab[dw];
        y = lds_tab[dw + 1];
    };
    uint32_t lo[NS], hi[NS];
    if (a.dir8 == 2u) {  // two-level, 4-bit counts (table.hpp kDir4GroupShift)
        uint32_t b[NS], w0[NS], w1[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const uint32_t g = t[s] >> kDir4GroupShift;
            b[s] = lds_tab[dir[s] + g];
            lds2(d16[s] + 2u * g, w0[s], w1[s]);  // one ds_read_b64 (8-byte aligned pair)
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) nib_bounds(b[s], w0[s], w1[s], t[s], lo[s], hi[s]);
    } else if (a.dir8) {  // two-level, u8 offsets (table.hpp kDir8GroupShift)
        uint32_t b0[NS], b1[NS], w0[NS], w1[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            lds2(dir[s] + (t[s] >> kDir8GroupShift), b0[s], b1[s]);
            lds2(d16[s] + (t[s] >> 2), w0[s], w1[s]);
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const uint32_t x = __builtin_amdgcn_alignbit(w1[s], w0[s], (t[s] & 3u) * 8u);
            lo[s] = b0[s] + (x & 0xFFu);
            hi[s] = (((t[s] + 1u) & ((1u << kDir8GroupShift) - 1u)) == 0u ? b1[s] : b0[s]) + ((x >> 8) & 0xFFu);
        }
    } else if (a.dir16) {  // two-level, u16 offsets
        uint32_t b0[NS], b1[NS], w0[NS], w1[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            lds2(dir[s] + (t[s] >> kDir16GroupShift), b0[s], b1[s]);
            lds2(d16[s] + (t[s] >> 1), w0[s], w1[s]);
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const bool odd = (t[s] & 1u) != 0u;
            lo[s] = b0[s] + (odd ? w0[s] >> 16 : w0[s] & 0xFFFFu);
            hi[s] = (((t[s] + 1u) >> kDir16GroupShift) != (t[s] >> kDir16GroupShift) ? b1[s] : b0[s]) +
                    (odd ? w1[s] & 0xFFFFu : w0[s] >> 16);
        }
    } else {  // plain u32
#pragma unroll
        for (int s = 0; s < NS; ++s) lds2(dir[s] + t[s], lo[s], hi[s]);
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        st[s] = lo[s];
        ln[s] = mine ? hi[s] - lo[s] : 0u;
    }
}

// `prefetch()` is called once, in the first pass, after the tests of its
// IPv6 round and first IPv4 window: the kernel issues the next batch's packet
// loads there (load mode 6) — younger than every entry load of the pass, so
// no test waits for them (vmcnt counts in order), and into registers the
// first window's entries have just freed.
// Timing probes (experiment builds only: make EXTRA=-DNFFACL_EXP_PIPE=k;
// verdicts wrong by design): 1 entry loads from one line (no gather
// traffic), 2 no candidate tests, 3 no marks / scans (every candidate owned
// by lane 0, entries from its stream number), 4 no directory lookups (one
// candidate per slot per packet).
#ifndef NFFACL_EXP_PIPE
#define NFFACL_EXP_PIPE 0
#endif
// 1: one mark pass per pass, marks carrying entry offsets (round 6); 0: the
// round-5 windows (marks + deltas per window), kept for A/B builds
#ifndef NFFACL_PIPE_ONEMARK
#define NFFACL_PIPE_ONEMARK 1
#endif

template <int NS, class PF>
__device__ __forceinline__ uint32_t classify_flat_pipe(const IndexedArgs &a, const Fields &f, FlatScratch<4> &W,
                                                       uint32_t lane, PF &&prefetch) {
    const bool v6 = f.is6;
    const uint32_t ks = __builtin_bswap32(f.s[0]), kd = __builtin_bswap32(f.t[0]);
    // list bounds, family streams: recomputed by every pass (a second pass
    // is rare: > 7 IPv4 rounds or > 1 IPv6 round in a batch), so that they
    // are dead while a pass's entry loads are in flight
    uint32_t st[NS], ln[NS], off = 0, T4 = 0, T6 = 0;
    auto streams = [&]() {
        if (NFFACL_EXP_PIPE == 4) {
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                st[s] = (f.t[0] >> (4 * s)) & 1023u;
                ln[s] = f.is4 || f.is6 ? 1u : 0u;
            }
        } else {
            flat_bounds_lds<NS>(a, f, st, ln);
        }
        uint32_t total = 0;
#pragma unroll
        for (int s = 0; s < NS; ++s) total += ln[s];
        const uint32_t t4 = v6 ? 0u : total, t6 = v6 ? total : 0u;
        const uint32_t i4 = wave_incl_sum(t4), i6 = wave_incl_sum(t6);
        T4 = __builtin_amdgcn_readlane(i4, 63);
        T6 = __builtin_amdgcn_readlane(i6, 63);
        off = v6 ? i6 - t6 : i4 - t4;  // this packet's first candidate in its family's stream
    };
    W.best[lane] = ~0ull;
    const uint8_t *tab8 = reinterpret_cast<const uint8_t *>(a.tab);
#if NFFACL_PIPE_ONEMARK
    // Round 6: ONE mark pass per pass for both families.  A mark carries its
    // list's entry offset instead of its window position:
    //   mark = owner lane << 26 | slot << 23 | (st - so + 2^22) mod 2^23
    // (ascending in stream order, as the prefix max needs; never 0), so the
    // candidate at stream number k reads its entry at family-relative
    // (mark mod 2^23) - 2^22 + k without a delta array — whose 1 KiB now
    // holds marks: 512 positions, the IPv4 window's 448 (7 rounds) at 0..447
    // and the IPv6 round's 64 at 448..511, marked together.  The owner's
    // protocol comes by one more ds_bpermute.  (Entry numbers < 2^22 per
    // family: indexed_launch.)
    uint32_t *const M = reinterpret_cast<uint32_t *>(&W);  // W.mark[256] + W.delta[256], contiguous
    const bool odd = (lane & 1u) != 0u;                    // (pair gathers)
    static_assert(sizeof(W.mark) + sizeof(W.delta) == 512 * sizeof(uint32_t), "512 marks");
    constexpr uint32_t kBias = 1u << 22, kOffMask = (1u << 23) - 1u;
    constexpr uint32_t kW4 = 448u, kP6 = 448u;  // IPv4 window length; the IPv6 round's first position
    auto mark_all = [&](uint32_t w4, uint32_t w6) {
        if (NFFACL_EXP_PIPE == 3) return;
        wave_lds_sync();  // (the previous pass's mark reads come first)
#pragma unroll
        for (int j = 0; j < 8; ++j) M[64 * j + lane] = 0u;
        wave_lds_sync();
        const uint32_t w = v6 ? w6 : w4, lim = v6 ? 64u : kW4, pb = v6 ? kP6 : 0u;
        uint32_t so = off;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if (ln[s] != 0u && so < w + lim && so + ln[s] > w)
                M[pb + (so > w ? so - w : 0u)] =
                    lane << 26 | static_cast<uint32_t>(s) << 23 | ((st[s] - so + kBias) & kOffMask);
            so += ln[s];
        }
        wave_lds_sync();
    };
    // Locate rounds j0 .. j0 + RR - 1 of the family window marked at pb,
    // continuing the prefix max from `carry`, and issue their entry loads
    // (lanes past the stream load the table's first bytes, untested).
    // mk[j] = the candidate's mark (its owner lane in bits 26..31).
    auto locate = [&](uint32_t pb, uint32_t w, uint32_t T, uint32_t j0, uint32_t &carry, auto six, auto rr,
                      uint32_t (&mk)[4], u32x3 (&A)[4], u32x3 (&B)[4], u32x3 &C, u32x3 &D) {
        constexpr bool SIX = decltype(six)::value;
        constexpr uint32_t ent_bytes = 4u * (SIX ? kHybEnt6Dwords : kHybEnt4Dwords);
        constexpr int RR = decltype(rr)::value;
        static_assert(!SIX || RR == 1, "IPv6 rounds: one per pass");
        const uint32_t fb4 = 4u * (SIX ? a.f6.off_ent_base : a.f4.off_ent_base);
        uint32_t scan[RR];
#pragma unroll
        for (int j = 0; j < RR; ++j)
            scan[j] = NFFACL_EXP_PIPE == 3 ? kBias : wave_incl_max(M[pb + 64u * (j0 + j) + lane]);
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            const uint32_t m = max(scan[j], carry);
            carry = __builtin_amdgcn_readlane(m, 63);
            mk[j] = m;
            const uint32_t k = w + 64u * (j0 + j) + lane;
            // family-relative entry number (< 2^22 for every valid k)
            const uint32_t en = (m & kOffMask) - kBias + k;
            uint32_t o = k < T ? fb4 + __umul24(en, ent_bytes) : 0u;
            if (NFFACL_EXP_PIPE == 1) o = 4u * a.f4.off_ent_base;
            if (NFFACL_EXP_PIPE == 3) o = 4u * a.f4.off_ent_base + __umul24(k & 4095u, ent_bytes);
            if (NFFACL_PAIR_GATHER) {  // unpacked by the round's test
                uint32_t oe, od;
                pair_offsets(o, odd, oe, od);
                const uint32_t *xe = reinterpret_cast<const uint32_t *>(tab8 + oe);
                const uint32_t *xd = reinterpret_cast<const uint32_t *>(tab8 + od);
                A[j] = ld3(xe);
                B[j] = ld3(xd);
                if constexpr (SIX) {
                    C = ld3(xe + 6);
                    D = ld3(xd + 6);
                }
            } else {
                const uint32_t *e = reinterpret_cast<const uint32_t *>(tab8 + o);
                A[j] = ld3(e);
                B[j] = ld3(e + 3);
                if constexpr (SIX) {
                    C = ld3(e + 6);
                    D = ld3(e + 9);
                }
            }
        }
    };
    // Test round j of a window: the owner packet's fields by ds_bpermute;
    // a passing candidate posts (rule index << 32 | output code) to the
    // owner's LDS minimum.
    auto post = [&](bool pass, uint32_t o, const u32x3 &A, const u32x3 &B) {
        if (NFFACL_EXP_PIPE == 2) {  // keep the loads alive without testing: one cheap use
            if ((A.x ^ B.z) == 0x5A5A5A5Au) W.best[lane] = 0u;
            return;
        }
        if (pass)
            atomicMin(reinterpret_cast<unsigned long long *>(&W.best[o]),
                      static_cast<unsigned long long>(A.z >> kEntIndexShift) << 32 | (B.z >> kHybOutShift));
    };
    auto test4 = [&](uint32_t w, uint32_t j0, auto rr, const uint32_t (&mk)[4], const u32x3 (&A)[4],
                     const u32x3 (&B)[4]) {
        constexpr int RR = decltype(rr)::value;
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            const uint32_t o = mk[j] >> 26;
            const uint32_t oks = bperm(ks, o), okd = bperm(kd, o), opt = bperm(f.ports, o), opr = bperm(f.proto, o);
            const bool valid = w + 64u * (j0 + j) + lane < T4;
            u32x3 ea = A[j], eb = B[j];
            if (NFFACL_PAIR_GATHER) pair_unpack(odd, ea, eb);
            const bool pass = valid & !hyb_miss(ea, eb, oks, okd, opr & 0xFFu, opt);
            post(pass, o, ea, eb);
        }
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    // One pass: one mark pass, then up to one IPv6 round from w6 and IPv4
    // rounds 0 .. R0 - 1 (<= 4) and R0 .. R0 + R1 - 1 (<= 3) from w4, issued
    // and tested in classify_flat_pipe's order (IPv6 round and first IPv4
    // rounds issued, IPv6 tested, the last IPv4 rounds issued, IPv4 tested).
    auto pass = [&](uint32_t w4, uint32_t w6, bool do6, auto r0, auto r1) {
        constexpr int R0 = decltype(r0)::value, R1 = decltype(r1)::value;
        uint32_t mk6[4], mkA[4], mkB[4];
        u32x3 A6[4], B6[4], C6, D6, AA[4], BA[4], AB[4], BB[4], cd;
        mark_all(w4, w6);
        uint32_t c6 = 0, c4 = 0;
        if (do6) locate(kP6, w6, T6, 0u, c6, std::true_type{}, I1{}, mk6, A6, B6, C6, D6);
        if constexpr (R0 > 0) locate(0u, w4, T4, 0u, c4, std::false_type{}, r0, mkA, AA, BA, cd, cd);
        if (do6) {  // the IPv6 round: every lane's address words 1..3 against its owner's
            const uint32_t o = mk6[0] >> 26;
            const uint32_t oks = bperm(ks, o), okd = bperm(kd, o), opt = bperm(f.ports, o), opr = bperm(f.proto, o);
            uint32_t os[4] = {0, 0, 0, 0}, ot[4] = {0, 0, 0, 0};
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                os[q] = bperm(__builtin_bswap32(f.s[q]), o);
                ot[q] = bperm(__builtin_bswap32(f.t[q]), o);
            }
            const bool valid = w6 + lane < T6;
            if (NFFACL_PAIR_GATHER) {
                pair_unpack(odd, A6[0], B6[0]);
                pair_unpack(odd, C6, D6);
            }
            // (one combined miss: no short-circuit branch)
            const bool m4 = hyb_miss(A6[0], B6[0], oks, okd, opr & 0xFFu, opt);
            const bool m6 = hyb_miss6(C6, D6, B6[0].z, os, ot);
            const bool miss6 = m4 || m6;
            const bool pass6 = valid & !miss6;
            post(pass6, o, A6[0], B6[0]);
        }
        if constexpr (R1 > 0) locate(0u, w4, T4, static_cast<uint32_t>(R0), c4, std::false_type{}, r1, mkB, AB, BB, cd, cd);
        if constexpr (R0 > 0) test4(w4, 0u, r0, mkA, AA, BA);
        if (w4 == 0u) prefetch();  // (the first pass)
        if constexpr (R1 > 0) test4(w4, static_cast<uint32_t>(R0), r1, mkB, AB, BB);
    };
#else
    // Mark the lists of family `fam6` overlapping the window [w, w + 64 RR):
    // mark[pos] = (owner lane << 19 | slot << 16 | pos << 8 | owner's protocol)
    // + 1 at the list's first position in the window, delta[pos] = byte
    // offset (from a.tab, mod 2^32) of the list's "candidate 0" entry.
    auto mark = [&](bool fam6, uint32_t w, auto rr) {
        constexpr int RR = decltype(rr)::value;
        if (NFFACL_EXP_PIPE == 3) return;
        wave_lds_sync();  // (the previous window's mark and delta reads come first)
#pragma unroll
        for (int j = 0; j < RR; ++j) W.mark[64 * j + lane] = 0u;
        wave_lds_sync();
        if (v6 == fam6) {
            const uint32_t ew = fam6 ? kHybEnt6Dwords : kHybEnt4Dwords;
            const uint32_t fb = fam6 ? a.f6.off_ent_base : a.f4.off_ent_base;
            uint32_t so = off;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                if (ln[s] != 0u && so < w + 64u * RR && so + ln[s] > w) {
                    const uint32_t pos = so > w ? so - w : 0u;
                    W.mark[pos] = (lane << 19 | static_cast<uint32_t>(s) << 16 | pos << 8 | (f.proto & 0xFFu)) + 1u;
                    // (signed 24-bit multiply, full rate: |st - so| < 2^23,
                    // table_consistent; v_mul_lo_u32 is quarter rate)
                    W.delta[pos] = (fb + static_cast<uint32_t>(__mul24(static_cast<int>(st[s] - so), static_cast<int>(ew))))
                                   << 2;
                }
                so += ln[s];
            }
        }
        wave_lds_sync();
    };
    // Locate the RR rounds of a marked window and issue their entry loads
    // (lanes past the stream load the table's first bytes, untested).
    // mk[j] = the candidate's mark - 1 (owner, protocol), k = stream number.
    auto locate = [&](uint32_t w, uint32_t T, auto six, auto rr, uint32_t (&mk)[4], u32x3 (&A)[4], u32x3 (&B)[4],
                      u32x3 &C, u32x3 &D) {
        constexpr bool SIX = decltype(six)::value;
        constexpr uint32_t ent_bytes = 4u * (SIX ? kHybEnt6Dwords : kHybEnt4Dwords);
        constexpr int RR = decltype(rr)::value;
        static_assert(!SIX || RR == 1, "IPv6 rounds: one per pass");
        uint32_t scan[RR];
#pragma unroll
        for (int j = 0; j < RR; ++j) scan[j] = NFFACL_EXP_PIPE == 3 ? 1u : wave_incl_max(W.mark[64 * j + lane]);
        uint32_t carry = 0;
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            const uint32_t m = max(scan[j], carry);
            if (j + 1 < RR) carry = __builtin_amdgcn_readlane(m, 63);
            mk[j] = m - 1u;
            const uint32_t k = w + 64u * j + lane;
            const uint32_t dp = W.delta[(mk[j] >> 8) & 0xFFu];
            uint32_t o = k < T ? dp + __umul24(k, ent_bytes) : 0u;
            if (NFFACL_EXP_PIPE == 1) o = 4u * a.f4.off_ent_base;
            if (NFFACL_EXP_PIPE == 3) {
                mk[j] = 0u;
                o = 4u * a.f4.off_ent_base + __umul24(k & 4095u, ent_bytes);
            }
            const uint32_t *e = reinterpret_cast<const uint32_t *>(tab8 + o);
            A[j] = ld3(e);
            B[j] = ld3(e + 3);
            if constexpr (SIX) {
                C = ld3(e + 6);
                D = ld3(e + 9);
            }
        }
    };
    // Test round j of a window: the owner packet's fields by ds_bpermute;
    // a passing candidate posts (rule index << 32 | output code) to the
    // owner's LDS minimum.
    auto post = [&](bool pass, uint32_t o, const u32x3 &A, const u32x3 &B) {
        if (NFFACL_EXP_PIPE == 2) {  // keep the loads alive without testing: one cheap use
            if ((A.x ^ B.z) == 0x5A5A5A5Au) W.best[lane] = 0u;
            return;
        }
        if (pass)
            atomicMin(reinterpret_cast<unsigned long long *>(&W.best[o]),
                      static_cast<unsigned long long>(A.z >> kEntIndexShift) << 32 | (B.z >> kHybOutShift));
    };
    auto test4 = [&](uint32_t w, auto rr, const uint32_t (&mk)[4], const u32x3 (&A)[4], const u32x3 (&B)[4]) {
        constexpr int RR = decltype(rr)::value;
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            const uint32_t o = mk[j] >> 19;
            const uint32_t oks = bperm(ks, o), okd = bperm(kd, o), opt = bperm(f.ports, o);
            const bool valid = w + 64u * j + lane < T4;
            const bool pass = valid & !hyb_miss(A[j], B[j], oks, okd, mk[j] & 0xFFu, opt);
            post(pass, o, A[j], B[j]);
        }
    };
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    using I4 = std::integral_constant<int, 4>;
    // One pass: up to one IPv6 round from w6 and IPv4 windows of R0 (<= 4)
    // and R1 (<= 3) rounds from w4 and w4 + 256.
    auto pass = [&](uint32_t w4, uint32_t w6, bool do6, auto r0, auto r1) {
        constexpr int R0 = decltype(r0)::value, R1 = decltype(r1)::value;
        uint32_t mk6[4], mkA[4], mkB[4];
        u32x3 A6[4], B6[4], C6, D6, AA[4], BA[4], AB[4], BB[4], cd;
        if (do6) {
            mark(true, w6, I1{});
            locate(w6, T6, std::true_type{}, I1{}, mk6, A6, B6, C6, D6);
        }
        if constexpr (R0 > 0) {
            mark(false, w4, r0);
            locate(w4, T4, std::false_type{}, r0, mkA, AA, BA, cd, cd);
        }
        if (do6) {  // the IPv6 round: every lane's address words 1..3 against its owner's
            const uint32_t o = mk6[0] >> 19;
            const uint32_t oks = bperm(ks, o), okd = bperm(kd, o), opt = bperm(f.ports, o);
            uint32_t os[4] = {0, 0, 0, 0}, ot[4] = {0, 0, 0, 0};
#pragma unroll
            for (int q = 1; q < 4; ++q) {
                os[q] = bperm(__builtin_bswap32(f.s[q]), o);
                ot[q] = bperm(__builtin_bswap32(f.t[q]), o);
            }
            const bool valid = w6 + lane < T6;
            // (one combined miss: no short-circuit branch)
            const bool m4 = hyb_miss(A6[0], B6[0], oks, okd, mk6[0] & 0xFFu, opt);
            const bool m6 = hyb_miss6(C6, D6, B6[0].z, os, ot);
            const bool miss6 = m4 || m6;
            const bool pass6 = valid & !miss6;
            post(pass6, o, A6[0], B6[0]);
        }
        if constexpr (R1 > 0) {
            mark(false, w4 + 256u, r1);
            locate(w4 + 256u, T4, std::false_type{}, r1, mkB, AB, BB, cd, cd);
        }
        if constexpr (R0 > 0) test4(w4, r0, mkA, AA, BA);
        if (w4 == 0u) prefetch();  // (the first pass)
        if constexpr (R1 > 0) test4(w4 + 256u, r1, mkB, AB, BB);
    };
#endif
    using I0 = std::integral_constant<int, 0>;
    uint32_t w4 = 0, w6 = 0;
    while (true) {
        streams();
        if (w4 >= T4 && w6 >= T6) {
            if (w4 == 0u && w6 == 0u) prefetch();  // a batch without candidates runs no pass
            break;
        }
        const uint32_t rem4 = T4 > w4 ? T4 - w4 : 0u;  // wave-uniform
        const bool do6 = w6 < T6;
        const uint32_t r = (rem4 + 63u) / 64u;  // IPv4 rounds left: 0..7 in this pass (more: next pass)
        if (r >= 7) pass(w4, w6, do6, I4{}, I3{});
        else if (r == 6) pass(w4, w6, do6, I4{}, I2{});
        else if (r == 5) pass(w4, w6, do6, I4{}, I1{});
        else if (r == 4) pass(w4, w6, do6, I4{}, I0{});
        else if (r == 3) pass(w4, w6, do6, I3{}, I0{});
        else if (r == 2) pass(w4, w6, do6, I2{}, I0{});
        else if (r == 1) pass(w4, w6, do6, I1{}, I0{});
        else pass(w4, w6, do6, I0{}, I0{});
        wave_lds_sync();
        w4 += 448u;
        w6 += 64u;
        if (w4 >= T4 && w6 >= T6) break;
    }
    uint64_t best = W.best[lane];  // ~0 or rule index << 32 | output code
    // rules with no selective key: wave-uniform scan in rule order per family
#pragma unroll
    for (int fam = 0; fam < 2; ++fam) {
        const FamArgs &fa = fam ? a.f6 : a.f4;
        const bool in_fam = fam ? f.is6 : f.is4;
        const uint32_t ew = fam ? kHybEnt6Dwords : kHybEnt4Dwords;
        for (uint32_t i = 0; i < fa.n_resid; ++i) {
            const uint32_t *e = a.tab + fa.off_resid + i * ew;
            const u32x3 RA = ld3(e), RB = ld3(e + 3);
            const uint32_t ri = RA.z >> kEntIndexShift;
            const bool want = in_fam && ri < uint32_t(best >> 32);
            if (!ballot(want)) break;  // residual list ascends too
            bool ok = want && !hyb_miss(RA, RB, ks, kd, f.proto, f.ports);
            if (fam && ballot(ok)) {
                uint32_t sb[4] = {0, 0, 0, 0}, tb[4] = {0, 0, 0, 0};
#pragma unroll
                for (int q = 1; q < 4; ++q) {
                    sb[q] = __builtin_bswap32(f.s[q]);
                    tb[q] = __builtin_bswap32(f.t[q]);
                }
                if (ok) ok = !hyb_miss6(ld3(e + 6), ld3(e + 9), RB.z, sb, tb);
            }
            best = ok ? (uint64_t(ri) << 32 | (RB.z >> kHybOutShift)) : best;
        }
    }
    const bool hit = best != ~0ull;
    uint32_t out = hit ? static_cast<uint32_t>(best) : 0u;
    const bool rd = hit && out == kHybOutEscape;
    if (ballot(rd)) {
        const uint32_t r = static_cast<uint32_t>(best >> 32);
        if (rd) out = a.tab[fam_sel(v6, a.f4.off_cold, a.f6.off_cold) + r];
        settle(out);
    }
    return out;
}

}  // namespace dev
}  // namespace nffacl
