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

#include "compile.hpp"
#include "devutil.hpp"
#include "engine.hpp"

namespace nffacl {

thread_local std::string g_last_error;

void set_last_error(const std::string &s) { g_last_error = s; }
const char *last_error() { return g_last_error.c_str(); }

namespace dev {

__device__ __forceinline__ uint32_t funnel16(uint32_t hi, uint32_t lo) {
    // ({hi,lo} >> 16)[31:0] : wire bytes 4k+2 .. 4k+5 as a LE dword
    return __builtin_amdgcn_alignbit(hi, lo, 16);
}

// Byte-swap each 16-bit half: LE dword of wire bytes [p0 p1 p2 p3] ->
// (p0<<8|p1) | (p2<<8|p3) << 16 = sport | dport << 16 (SwapBytesUint16,
// packet/packet.go:713-715, applied by l4ACL acl.go:511, 515).
__device__ __forceinline__ uint32_t swap_halves(uint32_t w) {
    return ((w & 0x00FF00FFu) << 8) | ((w >> 8) & 0x00FF00FFu);
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
template <bool REG_OPTS = false, class FarDwords>
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
    if (REG_OPTS) {
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
    if (f.is6) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            f.s[k] = funnel16(d[6 + k], d[5 + k]);
            f.t[k] = funnel16(d[10 + k], d[9 + k]);
        }
    } else {
        f.s[0] = funnel16(d[7], d[6]);
        f.t[0] = funnel16(d[8], d[7]);
#pragma unroll
        for (int k = 1; k < 4; ++k) { f.s[k] = 0; f.t[k] = 0; }
    }
}

// Dwords k and k+1 of a packet whose readable, zero-padded extent is `lim`
// bytes from `base` (4-byte aligned); bytes at or past `lim` read as 0.
__device__ __forceinline__ void far_dwords(const uint8_t *base, uint32_t lim, uint32_t k,
                                           uint32_t &lo, uint32_t &hi) {
    const uint32_t *p = reinterpret_cast<const uint32_t *>(base);
    auto masked = [&](uint32_t j) -> uint32_t {
        const int rem = static_cast<int>(lim) - static_cast<int>(4 * j);
        if (rem <= 0) return 0u;
        const uint32_t v = p[j];
        return rem >= 4 ? v : (v & ((1u << (8 * rem)) - 1u));
    };
    lo = masked(k);
    hi = masked(k + 1);
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
__device__ __forceinline__ void load_frames_rs(const uint8_t *__restrict__ frames, uint64_t ds, uint32_t lane,
                                               u32x4 (&v)[4]) {
    const uint32_t lo = static_cast<uint32_t>(ds), hi = static_cast<uint32_t>(ds >> 32);
    const uint32_t chunk = 16u * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int src = static_cast<int>((16u * j + (lane & 15u)) << 2);
        const uint32_t l = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(lo)));
        const uint32_t h = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(hi)));
        const uint64_t o = (uint64_t(h) << 32 | l) >> 16;
        v[j] = u32x4{0, 0, 0, 0};
        if (chunk < (l & 0xFFFFu)) v[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(frames + o) + (lane >> 4));
    }
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
    uint32_t generic;       // HYBRID flat forms: slots key on SlotArgs::f1/f2 (else slot s on field s)
    FamArgs f4, f6;
};

// Table placement (kernel template argument).
enum TableMode : int {
    kTabGlobal = 0,  // INDEXED, read through L1/L2/MALL
    kTabLds = 1,     // INDEXED, staged whole in LDS
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
};

extern __shared__ __attribute__((aligned(16))) uint32_t lds_tab[];

// Table accessors: the whole table staged in LDS, or read through L1/L2.
// ld4(i): i is a multiple of 4 (entries are 16-byte aligned, table.hpp) and is
// indexed in vector units so the compiler can emit one ds_read_b128 /
// global_load_dwordx4 (a byte-offset cast only gets split ds_read2_b32 pairs).
// List bounds dir[t], dir[t + 1] of a plain u32 directory (one ds_read2 /
// two dword loads).
template <class T>
__device__ __forceinline__ void bounds32(const T &tab, uint32_t dir, uint32_t t, uint32_t &lo, uint32_t &hi) {
    lo = tab.ld(dir + t);
    hi = tab.ld(dir + t + 1);
}

struct LdsTab {
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return lds_tab[i]; }
    __device__ __forceinline__ void bounds(uint32_t dir, uint32_t, uint32_t t, uint32_t &lo, uint32_t &hi,
                                           bool = false) const {
        bounds32(*this, dir, t, lo, hi);
    }
    __device__ __forceinline__ u32x4 ld4(uint32_t i) const {
        return reinterpret_cast<const u32x4 *>(lds_tab)[i >> 2];
    }
};
struct GlobalTab {
    const uint32_t *__restrict__ p;
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return p[i]; }
    __device__ __forceinline__ void bounds(uint32_t dir, uint32_t, uint32_t t, uint32_t &lo, uint32_t &hi,
                                           bool = false) const {
        bounds32(*this, dir, t, lo, hi);
    }
    __device__ __forceinline__ u32x4 ld4(uint32_t i) const {
        return reinterpret_cast<const u32x4 *>(p)[i >> 2];
    }
};
// HYBRID lane form: directories (ld) staged in LDS, entries (ld4) global.
struct SplitTab {
    const uint32_t *__restrict__ p;
    __device__ __forceinline__ uint32_t ld(uint32_t i) const { return lds_tab[i]; }
    // two-level directory (table.hpp): dir[t] = base[t >> 6] + dir16[t], or
    // with dir8 (wave-uniform) base[t >> 4] + dir8[t]
    __device__ __forceinline__ void bounds(uint32_t dir, uint32_t dir16, uint32_t t, uint32_t &lo, uint32_t &hi,
                                           bool dir8 = false) const {
        if (dir16 == 0u) {
            bounds32(*this, dir, t, lo, hi);
            return;
        }
        if (dir8) {
            const uint32_t g = t >> kDir8GroupShift;
            const uint32_t b0 = lds_tab[dir + g], b1 = lds_tab[dir + g + 1];                    // ds_read2
            const uint32_t w0 = lds_tab[dir16 + (t >> 2)], w1 = lds_tab[dir16 + (t >> 2) + 1];  // ds_read2
            const uint32_t x = __builtin_amdgcn_alignbit(w1, w0, (t & 3u) * 8u);  // bytes t, t + 1
            lo = b0 + (x & 0xFFu);
            hi = (((t + 1u) & ((1u << kDir8GroupShift) - 1u)) == 0u ? b1 : b0) + ((x >> 8) & 0xFFu);
            return;
        }
        const uint32_t g = t >> kDir16GroupShift;
        const uint32_t b0 = lds_tab[dir + g], b1 = lds_tab[dir + g + 1];                         // ds_read2
        const uint32_t w0 = lds_tab[dir16 + (t >> 1)], w1 = lds_tab[dir16 + (t >> 1) + 1];      // ds_read2
        const bool odd = (t & 1u) != 0u;
        lo = b0 + (odd ? w0 >> 16 : w0 & 0xFFFFu);
        hi = (((t + 1u) >> kDir16GroupShift) != g ? b1 : b0) + (odd ? w1 & 0xFFFFu : w0 >> 16);
    }
    __device__ __forceinline__ u32x4 ld4(uint32_t i) const {
        return reinterpret_cast<const u32x4 *>(p)[i >> 2];
    }
};

constexpr uint32_t kNone = 0xFFFFFFFFu;

// Mismatch bits of an entry's first 8 dwords (A = words 0..3, B = 4..7):
// address words, protocol (exact flag) and ports — acl.go:526-539 / 546-557
// with IPv6 restricted to the top 32 bits of each address.
__device__ __forceinline__ uint32_t entry_miss(const u32x4 &A, const u32x4 &B, const Fields &f) {
    const uint32_t proto = ((f.proto ^ B.x) & 0xFFu) & (0u - ((B.x >> 8) & 1u));
    return ((f.s[0] ^ A.x) & A.y) | ((f.t[0] ^ A.z) & A.w) | proto | port_miss(f.ports, B.y, B.z);
}

// Mismatch bits of the IPv6 extension words 8..19 (address words 1..3).
template <class T>
__device__ __forceinline__ uint32_t entry_miss_ext(const T &tab, uint32_t off, const Fields &f) {
    const u32x4 x = tab.ld4(off), y = tab.ld4(off + 4), z = tab.ld4(off + 8);
    // x = s1 s2 s3 sm1 | y = sm2 sm3 t1 t2 | z = t3 tm1 tm2 tm3
    return ((f.s[1] ^ x.x) & x.w) | ((f.s[2] ^ x.y) & y.x) | ((f.s[3] ^ x.z) & y.y) |
           ((f.t[1] ^ y.z) & z.y) | ((f.t[2] ^ y.w) & z.z) | ((f.t[3] ^ z.x) & z.w);
}

// First match over the four key slots of the lane's family, walked together:
// every iteration tests the next entry of every slot list, so the wave pays
// max(list lengths) table round trips, not their sum.  Loops have
// wave-uniform trip counts (ballots) and predicated bodies.
// U = list entries per slot per loop trip: all NS x U entry loads of a trip
// are issued before any is tested.
template <int NS, int U, class T>
__device__ __forceinline__ uint32_t classify_indexed(const T &tab, const IndexedArgs &a, const Fields &f) {
    const bool v6 = f.is6;
    const bool mine = f.is4 || f.is6;
    const uint32_t ew = v6 ? kEnt6Dwords : kEnt4Dwords;
    const uint32_t key[4] = {__builtin_bswap32(f.t[0]), __builtin_bswap32(f.s[0]), f.ports >> 16,
                             f.ports & 0xFFFFu};
    uint32_t c[NS], e[NS], base[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const SlotArgs &s4 = a.f4.slot[s], &s6 = a.f6.slot[s];
        const uint32_t shift = v6 ? s6.shift : s4.shift;
        const uint32_t dir = v6 ? s6.off_dir : s4.off_dir;
        base[s] = v6 ? s6.off_ent : s4.off_ent;
        const uint32_t t = key[s] >> shift;  // < n_buckets for any key: both reads in range
        uint32_t lo, hi;
        tab.bounds(dir, v6 ? s6.off_dir16 : s4.off_dir16, t, lo, hi, a.dir8 != 0u);
        c[s] = lo;
        e[s] = mine ? hi : lo;
    }
    uint32_t best = kNone, out = 0;
    while (true) {
        bool any = false;
#pragma unroll
        for (int s = 0; s < NS; ++s) any |= c[s] < e[s];
        if (!ballot(any)) break;
        u32x4 A[NS][U], B[NS][U];
#pragma unroll
        for (int s = 0; s < NS; ++s)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                // only lanes still walking this list load (a 16-byte load
                // costs the TA 16 cycles per 64 active lanes; LDS: -1.3 % on
                // C2, global: -4 % on C3, profiles/r1_masked)
                A[s][u] = B[s][u] = u32x4{0, 0, 0, 0};
                if (c[s] + u < e[s]) {
                    const uint32_t off = base[s] + (c[s] + u) * ew;
                    A[s][u] = tab.ld4(off);
                    B[s][u] = tab.ld4(off + 4);
                }
            }
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            bool go = true;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool act = go && c[s] + u < e[s];
                const uint32_t idx = B[s][u].x >> kEntIndexShift;
                const bool earlier = act && idx < best;
                bool pass = entry_miss(A[s][u], B[s][u], f) == 0u;
                const bool ext = v6 && earlier && pass;
                if (ballot(ext)) {
                    if (ext) pass = entry_miss_ext(tab, base[s] + (c[s] + u) * ew + 8, f) == 0u;
                }
                const bool take = earlier && pass;
                best = take ? idx : best;
                out = take ? B[s][u].w : out;
                // stop at a hit, or once the ascending list has passed `best`
                go = earlier && !pass;
            }
            c[s] = go ? c[s] + U : e[s];
        }
    }
    // rules with no selective key: wave-uniform scan in rule order per family
#pragma unroll
    for (int fam = 0; fam < 2; ++fam) {
        const FamArgs &fa = fam ? a.f6 : a.f4;
        const bool in_fam = fam ? f.is6 : f.is4;
        const uint32_t w = fam ? kEnt6Dwords : kEnt4Dwords;
        for (uint32_t i = 0; i < fa.n_resid; ++i) {
            const uint32_t off = fa.off_resid + i * w;
            const u32x4 A = tab.ld4(off), B = tab.ld4(off + 4);
            const uint32_t idx = B.x >> kEntIndexShift;
            const bool want = in_fam && idx < best;
            if (!ballot(want)) break;  // residual list ascends too
            bool pass = want && entry_miss(A, B, f) == 0u;
            if (fam && ballot(pass)) {
                if (pass) pass = entry_miss_ext(tab, off + 8, f) == 0u;
            }
            best = pass ? idx : best;
            out = pass ? B.w : out;
        }
    }
    return best != kNone ? out : 0u;
}

__device__ __forceinline__ void stage_table(const IndexedArgs &a) {
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a.tab);
    u32x4 *dst = reinterpret_cast<u32x4 *>(lds_tab);
    for (uint32_t i = threadIdx.x; i < a.stage_dwords / 4; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// ---- HYBRID (table.hpp "hybrid table") --------------------------------------

// Top-L-bits mask of a big-endian word, L in 0..32 (one 64-bit shift).
__device__ __forceinline__ uint32_t prefix_mask(uint32_t L) {
    return static_cast<uint32_t>(0xFFFFFFFF00000000ull >> L);
}

// 12-byte pieces of the exact flat-form entries (table.hpp): an IPv4 entry
// is two (the compiler issues dwordx4 + dwordx2), an IPv6 entry four.
typedef uint32_t u32x3 __attribute__((ext_vector_type(3), aligned(4)));

__device__ __forceinline__ u32x3 ld3(const uint32_t *__restrict__ p) { return *reinterpret_cast<const u32x3 *>(p); }

// Mismatch bits of an exact entry's first six words (both families): top
// address words under their prefix lengths (IPv6: capped at 32), protocol,
// ports — acl.go:526-539 / 546-557 for IPv4 completely, for IPv6 up to the
// low address words.  ks/kd: big-endian src/dst (top) words.
__device__ __forceinline__ uint32_t hyb_miss(const u32x3 &A, const u32x3 &B, uint32_t ks, uint32_t kd, uint32_t proto,
                                             uint32_t ports) {
    const uint32_t sl = min(B.z & 0xFFu, 32u), dl = min((B.z >> 8) & 0xFFu, 32u);
    const uint32_t pm = ((proto ^ A.z) & 0xFFu) & (0u - ((A.z >> 8) & 1u));
    return ((ks ^ A.x) & prefix_mask(sl)) | ((kd ^ A.y) & prefix_mask(dl)) | pm | port_miss(ports, B.x, B.y);
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

__device__ __forceinline__ uint32_t hyb_miss6(const u32x3 &C, const u32x3 &D, uint32_t lens, const uint32_t (&s)[4],
                                              const uint32_t (&t)[4]) {
    const uint32_t sl = lens & 0xFFu, dl = (lens >> 8) & 0xFFu;
    const uint32_t ps = 32u + first_diff96(s[1] ^ C.x, s[2] ^ C.y, s[3] ^ C.z);
    const uint32_t pd = 32u + first_diff96(t[1] ^ D.x, t[2] ^ D.y, t[3] ^ D.z);
    return (ps < sl ? 1u : 0u) | (pd < dl ? 1u : 0u);
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
    uint32_t mark[64 * R];   // window position -> (owner lane << 11 | slot << 8 | position) + 1, 0 = none
    uint32_t delta[64 * R];  // window position -> (entry number - candidate number) << 1 | IPv6
    uint64_t best[64];       // per packet (lane): lowest passing rule index << 32 | output code
};

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

template <int NS, int R, bool LDS_DIRS, bool UNCOND = false>
__device__ __forceinline__ uint32_t classify_flat(const IndexedArgs &a, const Fields &f, FlatScratch<R> &W,
                                                  uint32_t lane) {
    const bool v6 = f.is6;
    const bool mine = f.is4 || f.is6;
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
    if (LDS_DIRS && a.generic == 0u) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const SlotArgs &s4 = a.f4.slot[s], &s6 = a.f6.slot[s];
            const uint32_t key = s == kFDst ? kd : s == kFSrc ? ks : s == kFDport ? dport : s == kFSport ? sport : 0u;
            const uint32_t t = key >> (v6 ? s6.shift : s4.shift);
            uint32_t hi;
            SplitTab{a.tab}.bounds(v6 ? s6.off_dir : s4.off_dir, v6 ? s6.off_dir16 : s4.off_dir16, t, st[s], hi,
                                   a.dir8 != 0u);
            ln[s] = mine ? hi - st[s] : 0u;
        }
    } else {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const SlotArgs &s4 = a.f4.slot[s], &s6 = a.f6.slot[s];
        const uint32_t shift = v6 ? s6.shift : s4.shift;
        const uint32_t dir = v6 ? s6.off_dir : s4.off_dir;
        const uint32_t t = ((pick(v6 ? s6.f1 : s4.f1) >> shift) << (v6 ? s6.bits2 : s4.bits2)) |
                           (pick(v6 ? s6.f2 : s4.f2) >> (v6 ? s6.shift2 : s4.shift2));
        if (LDS_DIRS) {
            uint32_t hi;
            SplitTab{a.tab}.bounds(dir, v6 ? s6.off_dir16 : s4.off_dir16, t, st[s], hi, a.dir8 != 0u);
            ln[s] = mine ? hi - st[s] : 0u;
        } else {
            // generalized slots: a family's unused slots (f1 == kFZero) read nothing
            st[s] = 0u;
            ln[s] = 0u;
            if (mine && (v6 ? s6.f1 : s4.f1) != kFZero) {
                st[s] = a.tab[dir + t];
                ln[s] = a.tab[dir + t + 1] - st[s];
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
    const uint32_t proto_fam = f.proto | (v6 ? 0x100u : 0u);
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
                W.mark[pos] = ((lane << 11 | static_cast<uint32_t>(s) << 8) | pos) + 1u;
                W.delta[pos] = ((st[s] - so) << 1) | (v6 ? 1u : 0u);
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
        uint32_t owner[RR], idx[RR];
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
            owner[j] = (m - 1u) >> 11;
            const uint32_t dp = W.delta[(m - 1u) & 0xFFu];
            six[j] = (dp & 1u) != 0u;
            // UNCOND: lanes past the wave's candidates load entry 0 of the
            // IPv4 list (untested) instead of branching around the load
            // (profiles/r2_exact/uncond/)
            const uint32_t ent = !UNCOND || valid[j] ? k + static_cast<uint32_t>(static_cast<int32_t>(dp) >> 1) : 0u;
            const uint32_t *e = six[j] && (!UNCOND || valid[j]) ? E6 + ent * kHybEnt6Dwords : E4 + ent * kHybEnt4Dwords;
            if (UNCOND || valid[j]) {
                A[j] = ld3(e);
                B[j] = ld3(e + 3);
            } else {
                A[j] = B[j] = u32x3{0, 0, 0};
            }
            if (valid[j] && six[j]) {  // (C, D are read only for valid IPv6 candidates)
                C[j] = ld3(e + 6);
                D[j] = ld3(e + 9);
            }
        }
        bool pass[RR];
        bool any6 = false;
#pragma unroll
        for (int j = 0; j < RR; ++j) {
            // the owner packet's fields
            const uint32_t o = owner[j];
            const uint32_t oks = bperm(ks, o), okd = bperm(kd, o);
            const uint32_t opf = bperm(proto_fam, o), opt = bperm(f.ports, o);
            pass[j] = valid[j] && hyb_miss(A[j], B[j], oks, okd, opf & 0xFFu, opt) == 0u;
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
                    if (pass[j] && six[j]) pass[j] = hyb_miss6(C[j], D[j], B[j].z, os, ot) == 0u;
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
            const u32x3 RA = ld3(e), RB = ld3(e + 3);
            const uint32_t ri = RA.z >> kEntIndexShift;
            const bool want = in_fam && ri < uint32_t(best >> 32);
            if (!ballot(want)) break;  // residual list ascends too
            bool ok = want && hyb_miss(RA, RB, ks, kd, f.proto, f.ports) == 0u;
            if (fam && ballot(ok)) {
                uint32_t sb[4] = {0, 0, 0, 0}, tb[4] = {0, 0, 0, 0};
#pragma unroll
                for (int q = 1; q < 4; ++q) {
                    sb[q] = __builtin_bswap32(f.s[q]);
                    tb[q] = __builtin_bswap32(f.t[q]);
                }
                if (ok) ok = hyb_miss6(ld3(e + 6), ld3(e + 9), RB.z, sb, tb) == 0u;
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
        if (rd) out = a.tab[(v6 ? a.f6.off_cold : a.f4.off_cold) + r];
    }
    return out;
}

template <int NS, int TM>
__device__ __forceinline__ uint32_t classify_any(const IndexedArgs &a, const Fields &f) {
    if (TM == kTabFlat || TM == kTabFlat4) {
        constexpr int R = TM == kTabFlat4 ? 4 : 2;
        FlatScratch<R> *W = reinterpret_cast<FlatScratch<R> *>(lds_tab);
        const uint32_t lane = lane_id();
        return classify_flat<NS, R, false>(a, f, W[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)], lane);
    }
    if (TM == kTabFlatLds || TM == kTabFlatLds4 || TM == kTabFlatLds4U) {  // scratch after the staged directories (stage_dwords: multiple of 4)
        constexpr int R = TM == kTabFlatLds ? 2 : 4;
        FlatScratch<R> *W = reinterpret_cast<FlatScratch<R> *>(lds_tab + a.stage_dwords);
        const uint32_t lane = lane_id();
        return classify_flat<NS, R, true, TM == kTabFlatLds4U>(a, f, W[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)],
                                                               lane);
    }
    if constexpr (NS <= 4) {  // per-lane walks: the positional four slots
        if (TM == kTabLds) return classify_indexed<NS, 1>(LdsTab{}, a, f);
        if (TM == kTabSplit) return classify_indexed<NS, 1>(SplitTab{a.tab}, a, f);
        return classify_indexed<NS, 1>(GlobalTab{a.tab}, a, f);
    }
    return 0u;
}

// Grid-stride over 64-packet batches.
//  * rows (any stride): the next batch's 64-byte rows are loaded while the
//    current batch is classified (software pipelining, 16 VGPRs);
//  * COAL (stride == 64): lane-contiguous loads + quad transpose, lane l
//    classifying packet coal_packet(l) of its wave's batch; no register
//    prefetch (it would push the kernel past 64 VGPRs, i.e. below 8 waves per
//    SIMD) — 32 resident waves per CU keep 128 KiB of loads in flight.
template <int NS, int TM, int MODE>
__global__ void __launch_bounds__(1024)
k_indexed_slots(const uint8_t *__restrict__ slots, uint32_t stride, uint64_t n, IndexedArgs a,
                uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    if (TM == kTabLds || TM == kTabSplit || TM == kTabFlatLds || TM == kTabFlatLds4 || TM == kTabFlatLds4U) stage_table(a);
    const uint32_t lane = lane_id();
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t wave0 = uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = uint64_t(gridDim.x) * wpb * 64;
    constexpr bool RS = MODE == 4 || MODE == 5;  // lane-contiguous loads + permlane row swaps
    constexpr bool RSPF = MODE == 5;             // RS + the next batch's loads in flight (16 VGPRs)
    constexpr bool COAL = MODE != 0 && !RS;      // lane-contiguous loads + quad DPP transpose
    constexpr bool NT = MODE >= 2;
    constexpr bool PF = MODE == 3;  // coalesced + next-batch register prefetch
    const uint32_t mine = COAL ? coal_packet(lane) : lane;  // packet of this lane within the batch
    uint64_t base = wave0 * 64;
    uint32_t d[16];
    u32x4 nv[4];
    if (!COAL && !RS && base < n) load16(slots + (base + lane < n ? base + lane : 0) * stride, d);
    if (PF && base + 64 <= n) load_coal<NT>(slots + base * 64, lane, nv);
    if (RSPF && base + 64 <= n) load_rowswap<NT>(slots + base * 64, lane, nv);
    for (; base < n; base += step) {
        const uint64_t idx = base + mine;
        const bool live = idx < n;
        const uint8_t *pkt = slots + (live ? idx : 0) * stride;
        uint32_t cur[16];
        if (RS) {
            if (base + 64 <= n) {
                u32x4 cv[4];
                if (RSPF) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) cv[j] = nv[j];
                    const uint64_t nb = base + step;
                    if (nb + 64 <= n) load_rowswap<NT>(slots + nb * 64, lane, nv);
                } else {
                    load_rowswap<NT>(slots + base * 64, lane, cv);
                }
                rowswap_batch(cv, cur);
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
        // the streaming INDEXED kernel (C2) keeps the divergent far read
        // (the select chain cost it 2.6 %, round 1)
        constexpr bool REG = TM == kTabFlatLds || TM == kTabFlatLds4 || TM == kTabFlatLds4U;
        parse_fields<REG>(cur, live, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
            far_dwords(pkt, stride, k, lo, hi);
        }, a.flags);
        const uint32_t res = classify_any<NS, TM>(a, f);
        if (live && port_out) port_out[idx] = res;
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
}

template <int NS, int TM>
__global__ void __launch_bounds__(1024)
k_indexed_frames(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint64_t n,
                 IndexedArgs a, uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    if (TM == kTabLds || TM == kTabSplit || TM == kTabFlatLds || TM == kTabFlatLds4 || TM == kTabFlatLds4U) stage_table(a);
    const uint32_t lane = lane_id();
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t S = uint64_t(gridDim.x) * wpb * 64;  // grid stride in packets
    uint64_t base = (uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 64;
    if (base >= n) return;
    auto desc_at = [&](uint64_t b) -> uint64_t { return b + lane < n ? desc[b + lane] : 0; };
    // classify the batch at b whose descriptor is ds and first 64 bytes d
    auto classify_batch = [&](uint64_t b, uint64_t ds, uint32_t(&d)[16]) {
        const bool live = b + lane < n;
        const uint32_t len = static_cast<uint32_t>(ds & 0xFFFFu);
        const uint8_t *pkt = frames + (ds >> 16);
        // bytes past the frame read as 0; IMIX frames are all >= 64 bytes, so
        // the clip is skipped unless some lane of the wave holds a shorter one
        if (ballot(live && len < 64u)) clip16(d, len);
        Fields f;
        parse_fields<true>(d, live, f, [&](uint32_t k, uint32_t &lo, uint32_t &hi) {
            far_dwords(pkt, len, k, lo, hi);
        }, a.flags);
        const uint32_t res = classify_any<NS, TM>(a, f);
        store_verdicts(b, lane, live, res, port_out, permit_out);
    };
    // Software pipeline.  Always: the next batch's descriptors load while this
    // batch is classified (the frame load depends on them).  PF (per-lane
    // HYBRID walks, whose LDS directories hold the CU to 16 waves and so leave
    // VGPRs to spare): also the next batch's 64-byte frame lines, into the
    // other of two register buffers (ping-pong, no copies), and the
    // descriptors of the batch after.
    constexpr bool PF = TM == kTabSplit;  // (flat-LDS: +0.6 % on C3, profiles/r1_flat_lds/cold/)
    // (flat-LDS, round 2: one prefetch buffer with copies, 2 rounds — 124
    // VGPRs, no spill — ran 0.487 vs 0.469 ms on C3: the frame loads are not
    // what the walk waits on; profiles/r2_valu/pfab/)
    // Frame lines load cooperatively (load_frames_rs) and are assembled per
    // lane just before their batch is classified.
    auto run_batch = [&](uint64_t b, uint64_t ds, const u32x4(&v)[4]) {
        uint32_t d[16];
        rowswap_batch(v, d);
        classify_batch(b, ds, d);
    };
    if (PF) {
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
    } else {
        uint64_t ds_next = desc_at(base);
        for (; base < n; base += S) {
            const uint64_t ds = ds_next;
            ds_next = desc_at(base + S);
            u32x4 v[4];
            load_frames_rs(frames, ds, lane, v);
            run_batch(base, ds, v);
        }
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
    if (!env_knob("NFFACL_TUNE_COAL", 0, 5, v, set, err)) return false;
    if (set) t.coal = static_cast<int>(v);
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
    return CompileOptions::from_env(t.copt, err);
}

int upload_table(nffacl_engine *eng, const nffacl_rules &rules, TablePtr &out) {
    auto t = std::make_shared<DevTable>();
    std::string err;
    if (!compile_table(rules, eng->algo_req, eng->tune.copt, t->meta, err)) {
        set_last_error("compile: " + err);
        return NFFACL_ERR_INVALID_ARG;
    }
    HIP_TRY(hipSetDevice(eng->device));
    const hipError_t e = t->upload(&eng->home, t->meta.blob.data(), t->meta.blob.size());
    if (e != hipSuccess) {
        set_last_error(std::string("table upload: ") + hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? NFFACL_ERR_NOMEM : NFFACL_ERR_HIP;
    }
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
    if (m.algo == NFFACL_ALGO_HYBRID && (m.lds_dwords == 0 || m.idx4.entry_dwords == kHybEnt4Dwords))
        return m.idx4.entry_dwords == kHybEnt4Dwords && m.idx6.entry_dwords == kHybEnt6Dwords &&
               m.off_rec4 <= dw && m.off_rec6 <= dw &&
               size_t(m.lds_dwords) * sizeof(uint32_t) <= kHybLdsDirMaxBytes && m.lds_dwords <= dw;
    if (m.algo == NFFACL_ALGO_HYBRID)
        return size_t(m.lds_dwords) * sizeof(uint32_t) <= kLdsTableBytes && m.lds_dwords <= dw &&
               m.idx4.entry_dwords == kEnt4Dwords && m.idx6.entry_dwords == kEnt6Dwords;
    return m.idx4.entry_dwords == kEnt4Dwords && m.idx6.entry_dwords == kEnt6Dwords;
}

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
        return L;
    }
    if (t->meta.algo == NFFACL_ALGO_HYBRID) {
        staged = size_t(t->meta.lds_dwords) * sizeof(uint32_t);
        L.tm = dev::kTabSplit;
    } else {
        const size_t bytes = t->meta.blob.size() * sizeof(uint32_t);
        if (bytes <= kLdsTableBytes && tu.lds != 0) {
            L.tm = dev::kTabLds;
            staged = bytes;
        }
    }
    if (L.tm != dev::kTabGlobal) {
        L.block = 1024u;
        // lane form: one workgroup per CU (its VGPRs allow no second one)
        L.per_cu = L.tm == dev::kTabSplit
                       ? 1u
                       : static_cast<uint32_t>(std::max<size_t>(1, std::min<size_t>(2, kLdsBytes / std::max<size_t>(staged, 16))));
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
    if (TM == dev::kTabFlatLds || TM == dev::kTabFlatLds4 || TM == dev::kTabFlatLds4U)
        if (e == hipSuccess) e = allow_lds(dev::k_indexed_slots<NS, TM, 5>);
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
    auto with_ns = [&](auto nsc) {
        switch (tm) {
        case dev::kTabLds: f(nsc, std::integral_constant<int, dev::kTabLds>{}); break;
        case dev::kTabSplit: f(nsc, std::integral_constant<int, dev::kTabSplit>{}); break;
        case dev::kTabFlat: f(nsc, std::integral_constant<int, dev::kTabFlat>{}); break;
        case dev::kTabFlat4: f(nsc, std::integral_constant<int, dev::kTabFlat4>{}); break;
        case dev::kTabFlatLds: f(nsc, std::integral_constant<int, dev::kTabFlatLds>{}); break;
        case dev::kTabFlatLds4: f(nsc, std::integral_constant<int, dev::kTabFlatLds4>{}); break;
        case dev::kTabFlatLds4U: f(nsc, std::integral_constant<int, dev::kTabFlatLds4U>{}); break;
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
}

int prepare_kernels() {
    static std::once_flag once;
    static hipError_t err = hipSuccess;
    std::call_once(once, [] {
        for (int ns = 2; ns <= int(kMaxSlots); ++ns)
            for (int tm : {int(dev::kTabLds), int(dev::kTabSplit), int(dev::kTabFlatLds), int(dev::kTabFlatLds4),
                           int(dev::kTabFlatLds4U)}) {
                if (ns > 4 && tm != dev::kTabFlatLds && tm != dev::kTabFlatLds4 && tm != dev::kTabFlatLds4U)
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

template <int NS, int TM>
static void launch_slots_tm(int mode, const IndexedLaunch &L, uint32_t grid, hipStream_t stream,
                            const uint8_t *d_slots, uint32_t stride, uint64_t n, const dev::IndexedArgs &a,
                            uint32_t *d_port, uint64_t *d_permit) {
    const dim3 g(grid), b(L.block);
    const size_t lds = TM == dev::kTabGlobal ? 0 : L.lds_bytes;
    if constexpr (TM == dev::kTabFlatLds || TM == dev::kTabFlatLds4 || TM == dev::kTabFlatLds4U) {  // load modes 0, 4, 5
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
        const uint32_t grid = grid_for(eng, n, L.block, L.per_cu);
        const int mode = stride == 64 ? eng->tune.coal : 0;
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
        const uint32_t grid = grid_for(eng, n, L.block, L.per_cu);
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

}  // namespace nffacl
