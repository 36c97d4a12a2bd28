// l2.hip — HIP kernels (gfx950) for nff-go's L2 ACL: (*Packet).l2ACL,
// packet/acl.go:478-491, behind L2ACLPort / L2ACLPermit (acl.go:462-476).
//
// One wave64 = 64 consecutive packets, one packet per lane; each lane needs
// only the 16-byte line holding its Ethernet header (one load).
//  * LINEAR: records are wave-uniform and stream through the scalar data
//    cache; a ballot of still-undecided lanes ends the scan at the wave's
//    last first-match (the reference's `return rule.OutputNumber`).
//  * HASH: per rule shape both slots of a two-choice cuckoo table (see
//    l2.hpp); tables staged in LDS per workgroup when they fit, read through
//    L1/L2 otherwise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <type_traits>

#include "devutil.hpp"
#include "l2.hpp"

namespace nffacl {

namespace {

struct Masked {
    std::array<uint32_t, 4> v, m;  // pre-masked value, mask (m3 = EtherType mask, low 16 bits)
};

Masked masked_rule(const nffacl_l2_rule &r) {
    uint8_t val[12] = {0}, msk[12] = {0};
    if (r.daddr_not_any) {
        std::memcpy(val, r.daddr, 6);
        std::memset(msk, 0xff, 6);
    }
    if (r.saddr_not_any) {
        std::memcpy(val + 6, r.saddr, 6);
        std::memset(msk + 6, 0xff, 6);
    }
    Masked x;
    std::memcpy(x.v.data(), val, 12);
    std::memcpy(x.m.data(), msk, 12);
    // (rule.ID ^ SwapBytesUint16(EtherType)) & rule.IDMask (acl.go:486): the
    // big-endian EtherType compared with ID is, in wire-byte (LE) form, the
    // byte-swapped ID / IDMask.
    x.m[3] = static_cast<uint32_t>(((r.id_mask & 0xffu) << 8) | (r.id_mask >> 8));
    x.v[3] = static_cast<uint32_t>(((r.id & 0xffu) << 8) | (r.id >> 8));
    for (int k = 0; k < 4; ++k) x.v[k] &= x.m[k];
    return x;
}

// Per shape a two-choice cuckoo table at load <= 1/4 (one 16-byte slot per
// key: k0, k1, k2, k3 | rule index << 16).  Keys enter in ascending rule
// index, so the first owner of a key keeps it and later duplicates (shadowed
// rules) are dropped.  False if some key set cannot be placed within
// 8x its size (never seen; AUTO then compiles LINEAR).
bool build_cuckoo(const std::vector<Masked> &rules, const std::vector<nffacl_l2_rule> &eth,
                  const std::vector<std::array<uint32_t, 4>> &shapes,
                  const std::vector<std::vector<uint32_t>> &members, L2Compiled &c) {
    c.algo = NFFACL_ALGO_INDEXED;
    c.n_shapes = static_cast<uint32_t>(shapes.size());
    c.n_rules = static_cast<uint32_t>(rules.size());
    struct Slot {
        std::array<uint32_t, 4> k;
        uint32_t idx = kL2NoRule;
    };
    for (uint32_t s = 0; s < shapes.size(); ++s) {
        std::vector<uint32_t> keys;  // first owner of every distinct key, ascending
        {
            std::set<std::array<uint32_t, 4>> seen;
            for (uint32_t i : members[s])
                if (seen.insert(rules[i].v).second) keys.push_back(i);
        }
        uint32_t cap = 4;
        while (cap < 4 * keys.size()) cap <<= 1;
        std::vector<Slot> tab;
        bool placed_all = false;
        for (; !placed_all && cap <= 32 * std::max<size_t>(keys.size(), 4); cap <<= 1) {
            tab.assign(cap, Slot{});
            placed_all = true;
            for (uint32_t i : keys) {
                Slot cur{rules[i].v, i};
                uint32_t last = 0xFFFFFFFFu;  // the slot `cur` was just evicted from
                bool done = false;
                for (int kick = 0; kick < 500 && !done; ++kick) {
                    const uint32_t h = l2_hash(cur.k[0], cur.k[1], cur.k[2], cur.k[3]);
                    const uint32_t a0 = h & (cap - 1), a1 = l2_hash_alt(h) & (cap - 1);
                    if (tab[a0].idx == kL2NoRule) {
                        tab[a0] = cur;
                        done = true;
                    } else if (tab[a1].idx == kL2NoRule) {
                        tab[a1] = cur;
                        done = true;
                    } else {  // evict an occupant; it moves on to its other slot
                        const uint32_t victim = a0 == last ? a1 : a0;
                        std::swap(cur, tab[victim]);
                        last = victim;
                    }
                }
                if (!done) {
                    placed_all = false;
                    break;
                }
            }
        }
        if (!placed_all) return false;
        cap = static_cast<uint32_t>(tab.size());
        L2Shape &S = c.shapes[s];
        std::copy(shapes[s].begin(), shapes[s].end(), S.m);
        S.off = static_cast<uint32_t>(c.blob.size());
        S.cap_mask = cap - 1;
        for (const Slot &x : tab) {
            const uint32_t w[4] = {x.idx == kL2NoRule ? 0u : x.k[0], x.idx == kL2NoRule ? 0u : x.k[1],
                                   x.idx == kL2NoRule ? 0u : x.k[2],
                                   (x.idx == kL2NoRule ? 0u : x.k[3]) | (x.idx << 16)};
            c.blob.insert(c.blob.end(), w, w + 4);
        }
    }
    c.off_out = static_cast<uint32_t>(c.blob.size());
    for (uint32_t i = 0; i < rules.size(); ++i) c.blob.push_back(eth[i].output_number);
    while (c.blob.size() % 4) c.blob.push_back(0);
    return true;
}

}  // namespace

L2Compiled compile_l2(const std::vector<nffacl_l2_rule> &eth, int algo) {
    L2Compiled c;
    std::vector<Masked> rules;
    for (const nffacl_l2_rule &r : eth) {
        rules.push_back(masked_rule(r));
        const Masked &x = rules.back();
        if ((x.m[0] | x.m[1] | x.m[2] | x.m[3]) == 0) break;  // later rules unreachable
    }
    // shapes in order of first appearance
    std::vector<std::array<uint32_t, 4>> shapes;
    std::vector<std::vector<uint32_t>> members;
    for (uint32_t i = 0; i < rules.size(); ++i) {
        auto it = std::find(shapes.begin(), shapes.end(), rules[i].m);
        if (it == shapes.end()) {
            shapes.push_back(rules[i].m);
            members.emplace_back();
            it = shapes.end() - 1;
        }
        members[it - shapes.begin()].push_back(i);
    }
    const bool hash = algo != NFFACL_ALGO_LINEAR && shapes.size() <= kL2MaxShapes && rules.size() < kL2NoRule &&
                      build_cuckoo(rules, eth, shapes, members, c);
    if (!hash) {
        c = L2Compiled{};
        c.algo = NFFACL_ALGO_LINEAR;
        for (uint32_t i = 0; i < rules.size(); ++i) {
            const Masked &x = rules[i];
            const uint32_t w[kL2RecDwords] = {x.v[0], x.v[1], x.v[2], x.v[3] | (x.m[3] << 16),
                                              x.m[0], x.m[1], x.m[2], eth[i].output_number};
            c.blob.insert(c.blob.end(), w, w + kL2RecDwords);
        }
        c.n_rules = static_cast<uint32_t>(rules.size());
    }
    if (c.blob.empty()) c.blob.assign(kL2RecDwords, 0);  // keep a valid allocation
    return c;
}

int upload_l2(nffacl_l2engine *eng, const nffacl_l2rules &rules, L2TablePtr &out) {
    HIP_TRY(hipSetDevice(eng->device));
    auto t = std::make_shared<L2Table>();
    t->meta = compile_l2(rules.eth, eng->algo_req);
    const hipError_t e = t->upload(&eng->home, t->meta.blob.data(), t->meta.blob.size());
    if (e != hipSuccess) {
        set_last_error(std::string("L2 table upload: ") + hipGetErrorString(e));
        return e == hipErrorOutOfMemory ? NFFACL_ERR_NOMEM : NFFACL_ERR_HIP;
    }
    out = std::move(t);
    return NFFACL_OK;
}

namespace dev {

extern __shared__ __attribute__((aligned(16))) uint32_t l2_lds[];

// Packed shape descriptor: kind = EtherType mask | kL2PkDst | kL2PkSrc (MAC
// masks are whole addresses or nothing, acl.go:478-491).
struct L2Packed {
    uint32_t kind, off, cap_mask;
};
constexpr uint32_t kL2PkDst = 1u << 16, kL2PkSrc = 1u << 17;

struct L2Args {
    const uint32_t *tab;
    uint32_t tab_dwords;
    uint32_t n;        // LINEAR: records; HASH: shapes
    uint32_t off_out;  // HASH: OutputNumber per rule
    L2Packed pk[kL2MaxShapes];
};

__device__ __forceinline__ uint32_t classify_l2_linear(const uint32_t (&p)[4], bool live,
                                                       const uint32_t *__restrict__ rec, uint32_t n) {
    uint32_t res = 0;
    bool pend = live;
    for (uint32_t r = 0; r < n; ++r) {
        const uint32_t *R = rec + r * kL2RecDwords;
        const uint32_t m = ((p[0] ^ R[0]) & R[4]) | ((p[1] ^ R[1]) & R[5]) | ((p[2] ^ R[2]) & R[6]) |
                           ((p[3] ^ R[3]) & (R[3] >> 16));
        const bool take = pend && m == 0u;
        if (ballot(take)) {
            if (take) { res = R[7]; pend = false; }
            if (!ballot(pend)) break;
        }
    }
    return res;
}

// i: dword index, a multiple of 4 (ld4) — indexed in vector units so the
// compiler emits one ds_read_b128
template <bool LDS>
__device__ __forceinline__ u32x4 l2_ld4(const uint32_t *__restrict__ g, uint32_t i) {
    return LDS ? reinterpret_cast<const u32x4 *>(l2_lds)[i >> 2] : reinterpret_cast<const u32x4 *>(g)[i >> 2];
}
template <bool LDS>
__device__ __forceinline__ uint32_t l2_ld1(const uint32_t *__restrict__ g, uint32_t i) {
    return LDS ? l2_lds[i] : g[i];
}

// Shape s rebuilt from its packed descriptor (L2Args::pk).  The empty
// volatile asm keeps the rebuild inside the batch loop: hoisted for all
// eight shapes the masks would not fit the SGPR budget of eight waves per
// SIMD, while the packed words (3 SGPRs per shape) do.
__device__ __forceinline__ void unpack_shape(const L2Args &a, int s, uint32_t (&m)[4], uint32_t &off,
                                             uint32_t &cap) {
    uint32_t k = a.pk[s].kind;
    off = a.pk[s].off;
    cap = a.pk[s].cap_mask;
    asm volatile("" : "+s"(k), "+s"(off), "+s"(cap));
    m[0] = (k & kL2PkDst) ? 0xFFFFFFFFu : 0u;
    m[1] = ((k & kL2PkDst) ? 0x0000FFFFu : 0u) | ((k & kL2PkSrc) ? 0xFFFF0000u : 0u);
    m[2] = (k & kL2PkSrc) ? 0xFFFFFFFFu : 0u;
    m[3] = k & 0xFFFFu;
}

// Both cuckoo slots of every shape, no probe loop and no branch: a key is
// in one of its two slots or absent, and the lowest matching rule index over
// all shapes is the first match (empty slots carry kL2NoRule, which never
// wins).  Unrolled with constant shape indices, so the descriptors are
// loaded into SGPRs once per kernel.
template <bool LDS>
__device__ __forceinline__ uint32_t classify_l2_hash(const uint32_t (&p)[4], bool live, const L2Args &a) {
    uint32_t best = kL2NoRule;
#pragma unroll
    for (int s = 0; s < int(kL2MaxShapes); ++s) {
        if (uint32_t(s) >= a.n) break;
        uint32_t m[4], off, cap;
        unpack_shape(a, s, m, off, cap);
        const uint32_t k0 = p[0] & m[0], k1 = p[1] & m[1], k2 = p[2] & m[2], k3 = p[3] & m[3];
        const uint32_t h = l2_hash(k0, k1, k2, k3);
        const u32x4 r0 = l2_ld4<LDS>(a.tab, off + (h & cap) * 4u);
        const u32x4 r1 = l2_ld4<LDS>(a.tab, off + (l2_hash_alt(h) & cap) * 4u);
        const bool e0 = ((r0.x ^ k0) | (r0.y ^ k1) | (r0.z ^ k2) | ((r0.w & 0xFFFFu) ^ k3)) == 0u;
        const bool e1 = ((r1.x ^ k0) | (r1.y ^ k1) | (r1.z ^ k2) | ((r1.w & 0xFFFFu) ^ k3)) == 0u;
        best = min(best, e0 ? r0.w >> 16 : kL2NoRule);
        best = min(best, e1 ? r1.w >> 16 : kL2NoRule);
    }
    const bool hit = live && best != kL2NoRule;
    return hit ? l2_ld1<LDS>(a.tab, a.off_out + best) : 0u;
}

template <int ALGO, bool LDS>
__device__ __forceinline__ uint32_t classify_l2(const uint32_t (&p)[4], bool live, const L2Args &a) {
    if (ALGO == NFFACL_ALGO_LINEAR) return classify_l2_linear(p, live, a.tab, a.n);
    return classify_l2_hash<LDS>(p, live, a);
}

template <bool LDS>
__device__ __forceinline__ void l2_stage(const L2Args &a) {
    if (!LDS) return;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a.tab);
    u32x4 *dst = reinterpret_cast<u32x4 *>(l2_lds);
    for (uint32_t i = threadIdx.x; i < a.tab_dwords / 4; i += blockDim.x) dst[i] = src[i];
    __syncthreads();
}

// Two 1024-thread workgroups per CU (LDS mode) need 8 waves per SIMD: at most
// 64 VGPRs and 80 SGPRs (MI355X_MICROARCH.md: blocks per CU <=
// 800 / (ceil(sgpr/16)*16 + 16)).
// COAL (stride 64): a full batch's 4 KiB are loaded lane-contiguously
// (load_rowswap: one contiguous KiB per instruction, non-temporal) and each
// lane's header assembled with permlane swaps; otherwise one 16-byte row
// piece per lane.  Either way the next batch is loaded while this one is
// classified.
template <int ALGO, bool LDS, bool COAL>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_l2_slots(const uint8_t *__restrict__ slots, uint32_t stride, uint64_t n, L2Args a,
           uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    l2_stage<LDS>(a);
    const uint32_t lane = lane_id();
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t step = uint64_t(gridDim.x) * wpb * 64;
    uint64_t base = (uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 64;
    // next batch in flight: COAL full batches in nv[0..3], else the row piece in nv[0]
    u32x4 nv[4] = {};
    auto fetch = [&](uint64_t b) {
        if (COAL && b + 64 <= n)
            load_rowswap<true>(slots + b * 64, lane, nv);
        else
            nv[0] = *reinterpret_cast<const u32x4 *>(slots + (b + lane < n ? b + lane : 0) * stride);
    };
    if (base < n) fetch(base);
    for (; base < n; base += step) {
        uint32_t p[4];
        if (COAL && base + 64 <= n) {
            rowswap_chunk0(nv, p);
        } else {
            p[0] = nv[0].x; p[1] = nv[0].y; p[2] = nv[0].z; p[3] = nv[0].w;
        }
        if (base + step < n) fetch(base + step);
        const bool live = base + lane < n;
        store_verdicts(base, lane, live, classify_l2<ALGO, LDS>(p, live, a), port_out, permit_out);
    }
}

// Packed frames: desc = offset << 16 | length; bytes >= length read as 0.
template <int ALGO, bool LDS>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_l2_frames(const uint8_t *__restrict__ frames, const uint64_t *__restrict__ desc, uint64_t n, L2Args a,
            uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    l2_stage<LDS>(a);
    NFFACL_WAVE_LOOP(n) {
        const uint64_t idx = base + lane;
        const bool live = idx < n;
        const uint64_t ds = live ? desc[idx] : 0;
        // only frames with bytes are read: a 16-byte aligned load that starts
        // inside a frame stays inside that frame's page (no read past the
        // buffer, whatever follows the last frame)
        u32x4 v = u32x4{0, 0, 0, 0};
        if ((ds & 0xFFFFu) != 0u) v = *reinterpret_cast<const u32x4 *>(frames + (ds >> 16));
        uint32_t p[4] = {v.x, v.y, v.z, v.w};
        clip_dwords<4>(p, static_cast<uint32_t>(ds & 0xFFFFu));
        store_verdicts(base, lane, live, classify_l2<ALGO, LDS>(p, live, a), port_out, permit_out);
    }
}

}  // namespace dev

namespace {

constexpr size_t kL2LdsMax = 72 * 1024;  // two workgroups per CU keep their own copy

struct L2Launch {
    dev::L2Args a;
    bool lds;
    uint32_t block, grid;
    size_t lds_bytes;
};

L2Launch l2_plan(const nffacl_l2engine *eng, const L2Table *t, uint64_t n) {
    L2Launch L{};
    L.a.tab = t->d_blob;
    L.a.tab_dwords = static_cast<uint32_t>(t->meta.blob.size());
    const bool hash = t->meta.algo == NFFACL_ALGO_INDEXED;
    L.a.n = hash ? t->meta.n_shapes : t->meta.n_rules;
    L.a.off_out = t->meta.off_out;
    for (uint32_t s = 0; s < kL2MaxShapes; ++s) {
        const L2Shape &S = t->meta.shapes[s];
        L.a.pk[s] = dev::L2Packed{(S.m[3] & 0xFFFFu) | (S.m[0] ? dev::kL2PkDst : 0u) | (S.m[2] ? dev::kL2PkSrc : 0u),
                                  S.off, S.cap_mask};
    }
    L.lds_bytes = t->meta.blob.size() * sizeof(uint32_t);
    L.lds = hash && L.lds_bytes <= kL2LdsMax;
    L.block = L.lds ? 1024 : 256;
    const uint32_t per_cu = L.lds ? 2 : 8;
    const uint64_t blocks_needed = ((n + 63) / 64 * 64 + L.block - 1) / L.block;
    L.grid = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(blocks_needed, uint64_t(eng->num_cus) * per_cu)));
    return L;
}

}  // namespace

int l2_prepare_kernels() {
    static std::once_flag once;
    static hipError_t err = hipSuccess;
    std::call_once(once, [] {
        const void *k[3] = {reinterpret_cast<const void *>(dev::k_l2_slots<NFFACL_ALGO_INDEXED, true, false>),
                            reinterpret_cast<const void *>(dev::k_l2_slots<NFFACL_ALGO_INDEXED, true, true>),
                            reinterpret_cast<const void *>(dev::k_l2_frames<NFFACL_ALGO_INDEXED, true>)};
        for (const void *f : k) {
            hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kL2LdsMax));
            if (e != hipSuccess) err = e;
        }
    });
    if (err != hipSuccess) {
        set_last_error(std::string("hipFuncSetAttribute(L2 LDS): ") + hipGetErrorString(err));
        return NFFACL_ERR_HIP;
    }
    return NFFACL_OK;
}

int l2_launch_slots(nffacl_l2engine *eng, L2Table *t, const uint8_t *d_slots, uint32_t stride,
                    uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream) {
    if (n == 0) return NFFACL_OK;
    const L2Launch L = l2_plan(eng, t, n);
    const dim3 g(L.grid), b(L.block);
    const bool coal = stride == 64 && eng->coal;
    auto go = [&](auto algo_c, auto lds_c, auto coal_c) {
        hipLaunchKernelGGL((dev::k_l2_slots<decltype(algo_c)::value, decltype(lds_c)::value, decltype(coal_c)::value>),
                           g, b, decltype(lds_c)::value ? L.lds_bytes : 0, stream, d_slots, stride, n, L.a, d_port,
                           d_permit);
    };
    using lin = std::integral_constant<int, NFFACL_ALGO_LINEAR>;
    using hsh = std::integral_constant<int, NFFACL_ALGO_INDEXED>;
    using yes = std::true_type;
    using no = std::false_type;
    if (t->meta.algo == NFFACL_ALGO_LINEAR) {
        if (coal) go(lin{}, no{}, yes{}); else go(lin{}, no{}, no{});
    } else if (L.lds) {
        if (coal) go(hsh{}, yes{}, yes{}); else go(hsh{}, yes{}, no{});
    } else {
        if (coal) go(hsh{}, no{}, yes{}); else go(hsh{}, no{}, no{});
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(t->note_use(stream));
    return NFFACL_OK;
}

int l2_launch_frames(nffacl_l2engine *eng, L2Table *t, const uint8_t *d_frames, const uint64_t *d_desc,
                     uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream) {
    if (n == 0) return NFFACL_OK;
    const L2Launch L = l2_plan(eng, t, n);
    const dim3 g(L.grid), b(L.block);
    if (t->meta.algo == NFFACL_ALGO_LINEAR)
        hipLaunchKernelGGL((dev::k_l2_frames<NFFACL_ALGO_LINEAR, false>), g, b, 0, stream, d_frames, d_desc, n, L.a, d_port, d_permit);
    else if (L.lds)
        hipLaunchKernelGGL((dev::k_l2_frames<NFFACL_ALGO_INDEXED, true>), g, b, L.lds_bytes, stream, d_frames, d_desc, n, L.a, d_port, d_permit);
    else
        hipLaunchKernelGGL((dev::k_l2_frames<NFFACL_ALGO_INDEXED, false>), g, b, 0, stream, d_frames, d_desc, n, L.a, d_port, d_permit);
    HIP_TRY(hipGetLastError());
    HIP_TRY(t->note_use(stream));
    return NFFACL_OK;
}

}  // namespace nffacl
