// l2.hip — HIP kernels (gfx950) for nff-go's L2 ACL: (*Packet).l2ACL,
// packet/acl.go:478-491, behind L2ACLPort / L2ACLPermit (acl.go:462-476).
//
// One wave64 = 64 consecutive packets, one packet per lane; each lane needs
// only the 16-byte line holding its Ethernet header (one load).
//  * LINEAR: records are wave-uniform and stream through the scalar data
//    cache; a ballot of still-undecided lanes ends the scan at the wave's
//    last first-match (the reference's `return rule.OutputNumber`).
//  * HASH: per rule shape one hashed probe (see l2.hpp); tables staged in LDS
//    per workgroup when they fit, read through L1/L2 otherwise.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <map>
#include <string>

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
    const bool hash = algo != NFFACL_ALGO_LINEAR && shapes.size() <= kL2MaxShapes;
    if (!hash) {
        c.algo = NFFACL_ALGO_LINEAR;
        for (uint32_t i = 0; i < rules.size(); ++i) {
            const Masked &x = rules[i];
            const uint32_t w[kL2RecDwords] = {x.v[0], x.v[1], x.v[2], x.v[3] | (x.m[3] << 16),
                                              x.m[0], x.m[1], x.m[2], eth[i].output_number};
            c.blob.insert(c.blob.end(), w, w + kL2RecDwords);
        }
        c.n_rules = static_cast<uint32_t>(rules.size());
    } else {
        c.algo = NFFACL_ALGO_INDEXED;
        c.n_shapes = static_cast<uint32_t>(shapes.size());
        for (uint32_t s = 0; s < shapes.size(); ++s) {
            uint32_t buckets = 1;  // four slots each, at most half full
            while (buckets * kL2BucketSlots < 2 * members[s].size()) buckets <<= 1;
            const uint32_t slots = buckets * kL2BucketSlots;
            L2Shape &S = c.shapes[s];
            std::copy(shapes[s].begin(), shapes[s].end(), S.m);
            S.off = static_cast<uint32_t>(c.blob.size());
            S.off_key = S.off + slots;
            S.cap_mask = buckets - 1;
            S.first = members[s].front();
            c.blob.resize(c.blob.size() + size_t(slots) * (1 + kL2KeyDwords), 0);
            for (uint32_t i : members[s]) {  // ascending rule index: the first key owner wins
                const auto &v = rules[i].v;
                const uint32_t hv = l2_hash(v[0], v[1], v[2], v[3]);
                uint32_t bkt = hv & S.cap_mask;
                bool placed = false;
                while (!placed) {
                    for (uint32_t j = 0; j < kL2BucketSlots && !placed; ++j) {
                        const uint32_t slot = bkt * kL2BucketSlots + j;
                        uint32_t *fp = &c.blob[S.off + slot];
                        uint32_t *kr = &c.blob[S.off_key + size_t(slot) * kL2KeyDwords];
                        if (*fp == 0) {
                            *fp = hv | 1u;
                            kr[0] = v[0]; kr[1] = v[1]; kr[2] = v[2]; kr[3] = v[3];
                            kr[4] = i;
                            kr[5] = eth[i].output_number;
                            placed = true;
                        } else if (kr[0] == v[0] && kr[1] == v[1] && kr[2] == v[2] && kr[3] == v[3]) {
                            placed = true;  // shadowed by an earlier rule with the same key
                        }
                    }
                    bkt = (bkt + 1) & S.cap_mask;
                }
            }
        }
        std::sort(c.shapes, c.shapes + c.n_shapes,
                  [](const L2Shape &a, const L2Shape &b) { return a.first < b.first; });
        c.n_rules = static_cast<uint32_t>(rules.size());
    }
    if (c.blob.empty()) c.blob.assign(kL2RecDwords, 0);  // keep a valid allocation
    return c;
}

L2Table::~L2Table() {
    if (d_blob) (void)hipFree(d_blob);
}

int upload_l2(int device, const nffacl_l2rules &rules, int algo, L2Table *&out) {
    HIP_TRY(hipSetDevice(device));
    L2Table *t = new L2Table();
    t->meta = compile_l2(rules.eth, algo);
    const size_t bytes = t->meta.blob.size() * sizeof(uint32_t);
    hipError_t e = hipMalloc(reinterpret_cast<void **>(&t->d_blob), bytes);
    if (e == hipSuccess) e = hipMemcpy(t->d_blob, t->meta.blob.data(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        set_last_error(std::string("L2 table upload: ") + hipGetErrorString(e));
        delete t;
        return NFFACL_ERR_HIP;
    }
    out = t;
    return NFFACL_OK;
}

namespace dev {

extern __shared__ __attribute__((aligned(16))) uint32_t l2_lds[];

// Packed shape descriptor: kind = EtherType mask | kL2PkDst | kL2PkSrc (MAC
// masks are whole addresses or nothing, acl.go:478-491); key records follow
// the (cap_mask + 1) buckets.
struct L2Packed {
    uint32_t kind, off, cap_mask, first;
};
constexpr uint32_t kL2PkDst = 1u << 16, kL2PkSrc = 1u << 17;

struct L2Args {
    const uint32_t *tab;
    uint32_t tab_dwords;
    uint32_t n;  // LINEAR: records; HASH: shapes
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

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// i: dword index, a multiple of 4 (ld4) / 2 (ld2) — indexed in vector units
// so the compiler emits one ds_read_b128 / ds_read_b64
template <bool LDS>
__device__ __forceinline__ u32x4 l2_ld4(const uint32_t *__restrict__ g, uint32_t i) {
    return LDS ? reinterpret_cast<const u32x4 *>(l2_lds)[i >> 2] : reinterpret_cast<const u32x4 *>(g)[i >> 2];
}
template <bool LDS>
__device__ __forceinline__ u32x2 l2_ld2(const uint32_t *__restrict__ g, uint32_t i) {
    return LDS ? reinterpret_cast<const u32x2 *>(l2_lds)[i >> 1] : reinterpret_cast<const u32x2 *>(g)[i >> 1];
}
template <bool LDS>
__device__ __forceinline__ uint32_t l2_ld1(const uint32_t *__restrict__ g, uint32_t i) {
    return LDS ? l2_lds[i] : g[i];
}

// Shape lookups: one 16-byte fingerprint-bucket read per shape; a key record
// only on a fingerprint match; the next bucket only when this one is full and
// missed (rare at load <= 1/2).  Inactive lanes read bucket 0 (a broadcast).
template <bool LDS>
__device__ __forceinline__ void l2_lookup(const L2Shape &S, const uint32_t (&p)[4], bool go, const uint32_t *tab,
                                          uint32_t &best, uint32_t &res) {
    const uint32_t k0 = p[0] & S.m[0], k1 = p[1] & S.m[1], k2 = p[2] & S.m[2], k3 = p[3] & S.m[3];
    const uint32_t hv = l2_hash(k0, k1, k2, k3);
    const uint32_t f = hv | 1u;
    uint32_t bkt = go ? hv & S.cap_mask : 0u;
    while (true) {
        const u32x4 fp = l2_ld4<LDS>(tab, S.off + bkt * kL2BucketSlots);
        uint32_t mm = go ? (uint32_t(fp.x == f) | uint32_t(fp.y == f) << 1 | uint32_t(fp.z == f) << 2 |
                            uint32_t(fp.w == f) << 3)
                         : 0u;
        const bool has_free = (fp.x == 0u) | (fp.y == 0u) | (fp.z == 0u) | (fp.w == 0u);
        bool hit = false;
        while (ballot(mm != 0u)) {  // fingerprint matches (almost always one at most)
            const uint32_t j = mm ? static_cast<uint32_t>(__builtin_ctz(mm)) : 0u;
            const uint32_t at = S.off_key + (mm ? bkt * kL2BucketSlots + j : 0u) * kL2KeyDwords;
            const u32x4 e = l2_ld4<LDS>(tab, at);
            const bool eq = mm != 0u && ((e.x ^ k0) | (e.y ^ k1) | (e.z ^ k2) | (e.w ^ k3)) == 0u;
            if (eq) {
                const u32x2 io = l2_ld2<LDS>(tab, at + 4);  // rule index, OutputNumber
                if (io.x < best) { best = io.x; res = io.y; }
                hit = true;
            }
            mm = eq ? 0u : (mm & (mm - 1u));
        }
        go = go && !hit && !has_free;
        if (!ballot(go)) break;
        bkt = go ? (bkt + 1u) & S.cap_mask : 0u;
    }
}

// Shape s rebuilt from its packed descriptor (L2Args::pk).  The empty
// volatile asm keeps the rebuild inside the batch loop: hoisted for all
// eight shapes the masks would not fit the SGPR budget of eight waves per
// SIMD, while the packed words (4 SGPRs per shape) do.
__device__ __forceinline__ L2Shape unpack_shape(const L2Args &a, int s) {
    uint32_t k = a.pk[s].kind, off = a.pk[s].off, cap = a.pk[s].cap_mask, first = a.pk[s].first;
    asm volatile("" : "+s"(k), "+s"(off), "+s"(cap), "+s"(first));
    L2Shape S;
    S.m[0] = (k & kL2PkDst) ? 0xFFFFFFFFu : 0u;
    S.m[1] = ((k & kL2PkDst) ? 0x0000FFFFu : 0u) | ((k & kL2PkSrc) ? 0xFFFF0000u : 0u);
    S.m[2] = (k & kL2PkSrc) ? 0xFFFFFFFFu : 0u;
    S.m[3] = k & 0xFFFFu;
    S.off = off;
    S.cap_mask = cap;
    S.first = first;
    S.off_key = off + (cap + 1u) * kL2BucketSlots;
    return S;
}

// Shapes in ascending order of their first rule; a shape is skipped once
// every lane's match precedes it.  Unrolled with constant shape indices, so
// the descriptors are loaded into SGPRs once per kernel instead of by two
// scalar loads per shape and batch (each of which stalled the following LDS
// wait: lgkmcnt counts both).
template <bool LDS>
__device__ __forceinline__ uint32_t classify_l2_hash(const uint32_t (&p)[4], bool live, const L2Args &a) {
    uint32_t best = 0xFFFFFFFFu, res = 0;
#pragma unroll
    for (int s = 0; s < int(kL2MaxShapes); ++s) {
        if (s >= a.n) break;
        const L2Shape S = unpack_shape(a, s);
        const bool go = live && S.first < best;  // shapes ascend by first rule index
        if (!ballot(go)) break;
        l2_lookup<LDS>(S, p, go, a.tab, best, res);
    }
    return res;
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
template <int ALGO, bool LDS>
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_l2_slots(const uint8_t *__restrict__ slots, uint32_t stride, uint64_t n, L2Args a,
           uint32_t *__restrict__ port_out, uint64_t *__restrict__ permit_out) {
    l2_stage<LDS>(a);
    // grid-stride over 64-packet batches; the next batch's header line is
    // loaded while this one is classified (+10 % at 256 rules,
    // profiles/r1_l2_v3)
    const uint32_t lane = lane_id();
    const uint32_t wpb = blockDim.x >> 6;
    const uint64_t step = uint64_t(gridDim.x) * wpb * 64;
    uint64_t base = (uint64_t(blockIdx.x) * wpb + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * 64;
    auto header = [&](uint64_t b) {
        return *reinterpret_cast<const u32x4 *>(slots + (b + lane < n ? b + lane : 0) * stride);
    };
    u32x4 nv = base < n ? header(base) : u32x4{0, 0, 0, 0};
    for (; base < n; base += step) {
        const u32x4 v = nv;
        if (base + step < n) nv = header(base + step);
        const bool live = base + lane < n;
        const uint32_t p[4] = {v.x, v.y, v.z, v.w};
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
        const u32x4 v = *reinterpret_cast<const u32x4 *>(frames + (ds >> 16));
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
    for (uint32_t s = 0; s < kL2MaxShapes; ++s) {
        const L2Shape &S = t->meta.shapes[s];
        L.a.pk[s] = dev::L2Packed{(S.m[3] & 0xFFFFu) | (S.m[0] ? dev::kL2PkDst : 0u) | (S.m[2] ? dev::kL2PkSrc : 0u),
                                  S.off, S.cap_mask, S.first};
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
        const void *k[2] = {reinterpret_cast<const void *>(dev::k_l2_slots<NFFACL_ALGO_INDEXED, true>),
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

int l2_launch_slots(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_slots, uint32_t stride,
                    uint64_t n, uint32_t *d_port, uint64_t *d_permit, hipStream_t stream) {
    if (n == 0) return NFFACL_OK;
    const L2Launch L = l2_plan(eng, t, n);
    const dim3 g(L.grid), b(L.block);
    if (t->meta.algo == NFFACL_ALGO_LINEAR)
        hipLaunchKernelGGL((dev::k_l2_slots<NFFACL_ALGO_LINEAR, false>), g, b, 0, stream, d_slots, stride, n, L.a, d_port, d_permit);
    else if (L.lds)
        hipLaunchKernelGGL((dev::k_l2_slots<NFFACL_ALGO_INDEXED, true>), g, b, L.lds_bytes, stream, d_slots, stride, n, L.a, d_port, d_permit);
    else
        hipLaunchKernelGGL((dev::k_l2_slots<NFFACL_ALGO_INDEXED, false>), g, b, 0, stream, d_slots, stride, n, L.a, d_port, d_permit);
    HIP_TRY(hipGetLastError());
    return NFFACL_OK;
}

int l2_launch_frames(nffacl_l2engine *eng, const L2Table *t, const uint8_t *d_frames, const uint64_t *d_desc,
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
    return NFFACL_OK;
}

}  // namespace nffacl
