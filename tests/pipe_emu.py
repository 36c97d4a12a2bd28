"""Wave-level CPU model of the pipelined flat-LDS walk
(`classify_flat_pipe`, nff-go_amd/csrc/classify.hpp) over a compiled blob.

Test infrastructure (like oracle/): it restates, lane by lane and step by
step, what one 64-lane wave does to one batch — list bounds from the LDS
parameter block and 4-bit / u8 / u16 / plain directories (`flat_bounds_lds`),
the two family streams and their exclusive scans, the passes (one IPv6 round,
IPv4 windows of up to 4 + 3 rounds), the window marks and deltas in a
scratch that persists from batch to batch (stale contents included), the
prefix-max locate, byte-offset entry addresses mod 2^32 (lanes past the
stream load the table's first bytes), the owner fields by bpermute (lane =
address bits 7:2), the LDS minima, the residual scan and the output escape.
Verdicts are compared with the oracle by tests/test_pipe_walk.py; `trace`
records, per batch, the stream totals and the passes run, so a GPU
disagreement can be located in the walk (pass, window, round).

Semantics restated: first match in rule order, /root/reference/packet/acl.go:522-565.
"""
import numpy as np

ENT4, ENT6 = 6, 12          # table.hpp kHybEnt4Dwords / kHybEnt6Dwords
IDX_SHIFT, OUT_SHIFT = 9, 16
OUT_ESCAPE = 0xFFFF
PARAM_DWORDS = 4            # table.hpp kFlatParamDwords
M32 = 0xFFFFFFFF


def slot_fields(slots: np.ndarray, n: int, stride: int = 64):
    """Fields of dense slots as parse_fields sees them (no VLAN; bytes past
    the slot read 0): is4, is6, ks/kd (big-endian top address words), the
    IPv6 words 1..3, proto, ports = sport | dport << 16."""
    p = np.zeros((n, stride + 64), np.uint32)
    p[:, :stride] = slots.reshape(n, stride)[:, :stride]
    rows = np.arange(n)
    be = lambda o: p[:, o] << 24 | p[:, o + 1] << 16 | p[:, o + 2] << 8 | p[:, o + 3]  # noqa: E731
    is4 = (p[:, 12] == 0x08) & (p[:, 13] == 0x00)
    is6 = (p[:, 12] == 0x86) & (p[:, 13] == 0xDD)
    l4 = np.where(is6, 54, 14 + 4 * (p[:, 14] & 0xF))
    sport = p[rows, l4] << 8 | p[rows, l4 + 1]
    dport = p[rows, l4 + 2] << 8 | p[rows, l4 + 3]
    s = [np.where(is6, be(22 + 4 * q), be(26) if q == 0 else 0) for q in range(4)]
    t = [np.where(is6, be(38 + 4 * q), be(30) if q == 0 else 0) for q in range(4)]
    proto = np.where(is6, p[:, 20], p[:, 23])
    return dict(is4=is4, is6=is6, s=np.stack(s).astype(np.uint64), t=np.stack(t).astype(np.uint64),
                proto=proto.astype(np.uint64), ports=(sport | dport << 16).astype(np.uint64))


def _u16(x, half):
    return (int(x) >> half) & 0xFFFF


def bounds(blob, info, ns, ks, kd, sport, dport, v6, dir8, dir16):
    """flat_bounds_lds for one lane: (st[ns], ln-before-`mine`[ns])."""
    half = 16 if v6 else 0
    st, hi_ = [], []
    for s in range(ns):
        P = blob[info.off_params + PARAM_DWORDS * s: info.off_params + PARAM_DWORDS * (s + 1)]
        shift = _u16(P[0], half)
        d = _u16(P[1], half)
        d16 = _u16(P[2], half)
        if s < 4:
            key = (kd, ks, dport, sport)[s]
            t = key >> (shift & 31)  # v_lshrrev_b32: the shift's low 5 bits
        else:
            fine = _u16(P[3], half)
            addr = ks if s & 1 else kd
            port = dport if s < 6 else sport
            t = (((addr >> (shift & 31)) << (fine & 0xFF)) | (port >> ((fine >> 8) & 31))) & M32
        if dir8 == 2:
            g = t >> 4
            b = int(blob[d + g])
            x = int(blob[d16 + 2 * g]) | int(blob[d16 + 2 * g + 1]) << 32
            j = t & 15
            lo = b + sum((x >> (4 * i)) & 15 for i in range(j))
            hi = lo + ((x >> (4 * j)) & 15)
        elif dir8 == 1:
            b0, b1 = int(blob[d + (t >> 4)]), int(blob[d + (t >> 4) + 1])
            w = int(blob[d16 + (t >> 2)]) | int(blob[d16 + (t >> 2) + 1]) << 32
            x = (w >> ((t & 3) * 8)) & M32
            lo = b0 + (x & 0xFF)
            hi = (b1 if ((t + 1) & 15) == 0 else b0) + ((x >> 8) & 0xFF)
        elif dir16:
            b0, b1 = int(blob[d + (t >> 6)]), int(blob[d + (t >> 6) + 1])
            w0, w1 = int(blob[d16 + (t >> 1)]), int(blob[d16 + (t >> 1) + 1])
            odd = t & 1
            lo = b0 + ((w0 >> 16) if odd else (w0 & 0xFFFF))
            hi = (b1 if ((t + 1) >> 6) != (t >> 6) else b0) + ((w1 & 0xFFFF) if odd else (w0 >> 16))
        else:
            lo, hi = int(blob[d + t]), int(blob[d + t + 1])
        st.append(lo & M32)
        hi_.append(hi & M32)
    return st, [(h - lo) & M32 for h, lo in zip(hi_, st)]


def _pmask(L):
    return (0xFFFFFFFF00000000 >> L) & M32


def _first_diff96(x1, x2, x3):
    clz = lambda x: 32 - x.bit_length()  # noqa: E731
    return clz(x1) if x1 else 32 + clz(x2) if x2 else 64 + clz(x3)


def _miss(A, B, ks, kd, proto, ports):
    sl, dl = min(B[2] & 0xFF, 32), min((B[2] >> 8) & 0xFF, 32)
    pm = ((proto ^ A[2]) & 0xFF) if (A[2] >> 8) & 1 else 0
    m = ((ks ^ A[0]) & _pmask(sl)) | ((kd ^ A[1]) & _pmask(dl)) | pm
    c = 0
    for sh in (0, 16):
        p, lo, hi = (ports >> sh) & 0xFFFF, (B[0] >> sh) & 0xFFFF, (B[1] >> sh) & 0xFFFF
        c |= min(max(p, lo), hi) << sh
    return m | (c ^ ports)


def _miss6(C, D, lens, s, t):
    sl, dl = lens & 0xFF, (lens >> 8) & 0xFF
    ps = 32 + _first_diff96(s[1] ^ C[0], s[2] ^ C[1], s[3] ^ C[2])
    pd = 32 + _first_diff96(t[1] ^ D[0], t[2] ^ D[1], t[3] ^ D[2])
    return (1 if ps < sl else 0) | (1 if pd < dl else 0)


ONEMARK = True  # classify_flat_pipe's round-6 form (NFFACL_PIPE_ONEMARK=1); False: round 5's windows


class Scratch:
    """One wave's FlatScratch<4> (persists across the wave's batches): the
    round-5 form's mark[256] / delta[256], or the round-6 form's 512 marks
    over the same bytes (M)."""

    def __init__(self, rng):
        self.mark = [int(x) for x in rng.integers(0, 1 << 32, 256, dtype=np.uint64)]
        self.delta = [int(x) for x in rng.integers(0, 1 << 32, 256, dtype=np.uint64)]
        self.M = self.mark + self.delta
        self.best = [int(x) for x in rng.integers(0, 1 << 63, 64, dtype=np.uint64)]


def walk_batch(blob, info, ns, F, base, n, W, trace=None, where=None):
    """classify_flat_pipe over packets base .. base + 63 (lanes past n: not
    live).  Returns 64 verdicts.  `where` (a dict) receives, per packet whose
    minimum came from the walk, where its winning candidate sat: (pass,
    window 'v6' / 'A' / 'B', round, candidate lane, stream number)."""
    tab_bytes = blob.view(np.uint8)
    dir8 = info_dir8(info)
    dir16 = info_dir16(info)
    live = [base + l < n for l in range(64)]
    idx = [base + l if live[l] else base for l in range(64)]
    is4 = [live[l] and bool(F["is4"][idx[l]]) for l in range(64)]
    is6 = [live[l] and bool(F["is6"][idx[l]]) for l in range(64)]
    ks = [int(F["s"][0][i]) for i in idx]
    kd = [int(F["t"][0][i]) for i in idx]
    sw = [[int(F["s"][q][i]) for q in range(4)] for i in idx]
    tw = [[int(F["t"][q][i]) for q in range(4)] for i in idx]
    proto = [int(F["proto"][i]) for i in idx]
    ports = [int(F["ports"][i]) for i in idx]
    f4, f6 = info.fam[0], info.fam[1]

    st = [None] * 64
    ln = [None] * 64
    for l in range(64):
        s_, l_ = bounds(blob, info, ns, ks[l], kd[l], ports[l] & 0xFFFF, ports[l] >> 16, is6[l], dir8, dir16)
        mine = is4[l] or is6[l]
        st[l] = s_
        ln[l] = [x if mine else 0 for x in l_]
    tot = [sum(ln[l]) & M32 for l in range(64)]
    t4 = [0 if is6[l] else tot[l] for l in range(64)]
    t6 = [tot[l] if is6[l] else 0 for l in range(64)]
    T4, T6 = sum(t4) & M32, sum(t6) & M32
    off = []
    a4 = a6 = 0
    for l in range(64):
        off.append(a6 if is6[l] else a4)
        a4 = (a4 + t4[l]) & M32
        a6 = (a6 + t6[l]) & M32
    for l in range(64):
        W.best[l] = (1 << 64) - 1
    passes = []

    def ld(o, k):
        o &= M32
        assert o % 4 == 0 and o + 4 * k <= tab_bytes.size, f"entry load outside the table: {o}"
        return [int(x) for x in blob[o // 4: o // 4 + k]]

    def mark(fam6, w, RR):
        for j in range(64 * RR):
            W.mark[j] = 0
        ew = ENT6 if fam6 else ENT4
        fb = f6.off_ent_base if fam6 else f4.off_ent_base
        for l in range(64):
            if is6[l] != fam6:
                continue
            so = off[l]
            for s in range(ns):
                if ln[l][s] != 0 and so < w + 64 * RR and so + ln[l][s] > w:
                    pos = so - w if so > w else 0
                    W.mark[pos] = ((l << 19 | s << 16 | pos << 8 | (proto[l] & 0xFF)) + 1) & M32
                    W.delta[pos] = (((fb + (st[l][s] - so) * ew) & M32) << 2) & M32
                so = (so + ln[l][s]) & M32

    def locate(w, T, six, RR):
        ent_bytes = 4 * (ENT6 if six else ENT4)
        out = []
        m = 0
        for j in range(RR):
            rnd = []
            for l in range(64):
                m = max(m, W.mark[64 * j + l])
                mk = (m - 1) & M32
                k = w + 64 * j + l
                dp = W.delta[(mk >> 8) & 0xFF]
                o = (dp + k * ent_bytes) & M32 if k < T else 0
                A, B = ld(o, 3), ld(o + 12, 3)
                C = ld(o + 24, 3) if six else None
                D = ld(o + 36, 3) if six else None
                rnd.append((mk, k, A, B, C, D))
            out.append(rnd)
        return out

    loc = {}

    def post(ok, o, A, B, at):
        if ok:
            v = (A[2] >> IDX_SHIFT) << 32 | (B[2] >> OUT_SHIFT)
            if v < W.best[o]:
                W.best[o] = v
                loc[o] = at

    def test(rounds, T, six, name):
        for j, rnd in enumerate(rounds):
            for l, (mk, k, A, B, C, D) in enumerate(rnd):
                o = (mk >> 19) & 63  # ds_bpermute: lane = byte address bits 7:2
                miss = _miss(A, B, ks[o], kd[o], mk & 0xFF, ports[o])
                if six:
                    miss |= _miss6(C, D, B[2], sw[o], tw[o])
                post(k < T and miss == 0, o, A, B, (len(passes) - 1, name, j, l, k))

    BIAS, OMASK = 1 << 22, (1 << 23) - 1

    def mark_all(w4, w6):
        """One mark pass: IPv4 lists over [w4, w4 + 448) at 0..447, IPv6 over
        [w6, w6 + 64) at 448..511; mark = lane << 26 | slot << 23 | (st - so + 2^22) mod 2^23."""
        for j in range(512):
            W.M[j] = 0
        for l in range(64):
            w, lim, pb = (w6, 64, 448) if is6[l] else (w4, 448, 0)
            so = off[l]
            for s in range(ns):
                if ln[l][s] != 0 and so < w + lim and so + ln[l][s] > w:
                    W.M[pb + (so - w if so > w else 0)] = (l << 26 | s << 23 | ((st[l][s] - so + BIAS) & OMASK)) & M32
                so = (so + ln[l][s]) & M32

    def locate1(pb, w, T, j0, carry, six, RR):
        ent_bytes = 4 * (ENT6 if six else ENT4)
        fb4 = 4 * (f6.off_ent_base if six else f4.off_ent_base)
        out = []
        for j in range(j0, j0 + RR):
            rnd = []
            m = carry
            for l in range(64):
                m = max(m, W.M[pb + 64 * j + l])
                k = w + 64 * j + l
                en = ((m & OMASK) - BIAS + k) & M32
                o = (fb4 + en * ent_bytes) & M32 if k < T else 0
                A, B = ld(o, 3), ld(o + 12, 3)
                C = ld(o + 24, 3) if six else None
                D = ld(o + 36, 3) if six else None
                rnd.append((m, k, A, B, C, D))
            carry = m  # readlane(m, 63)
            out.append(rnd)
        return out, carry

    def test1(rounds, T, six, name, j0):
        for jj, rnd in enumerate(rounds):
            for l, (mk, k, A, B, C, D) in enumerate(rnd):
                o = (mk >> 26) & 63
                miss = _miss(A, B, ks[o], kd[o], proto[o] & 0xFF, ports[o])
                if six:
                    miss |= _miss6(C, D, B[2], sw[o], tw[o])
                post(k < T and miss == 0, o, A, B, (len(passes) - 1, name, j0 + jj, l, k))

    w4 = w6 = 0
    while True:
        if w4 >= T4 and w6 >= T6:
            break
        rem4 = T4 - w4 if T4 > w4 else 0
        do6 = w6 < T6
        r = (rem4 + 63) // 64
        R0, R1 = (4, 3) if r >= 7 else (4, r - 4) if r >= 4 else (r, 0)
        passes.append((w4, w6, do6, R0, R1))
        if ONEMARK:
            mark_all(w4, w6)
            r6 = ra = rb = None
            c4 = 0
            if do6:
                r6, _ = locate1(448, w6, T6, 0, 0, True, 1)
            if R0:
                ra, c4 = locate1(0, w4, T4, 0, 0, False, R0)
            if do6:
                test1(r6, T6, True, 'v6', 0)
            if R1:
                rb, c4 = locate1(0, w4, T4, R0, c4, False, R1)
            if R0:
                test1(ra, T4, False, 'A', 0)
            if R1:
                test1(rb, T4, False, 'B', R0)
        else:
            r6 = ra = rb = None
            if do6:
                mark(True, w6, 1)
                r6 = locate(w6, T6, True, 1)
            if R0:
                mark(False, w4, R0)
                ra = locate(w4, T4, False, R0)
            if do6:
                test(r6, T6, True, 'v6')
            if R1:
                mark(False, w4 + 256, R1)
                rb = locate(w4 + 256, T4, False, R1)
            if R0:
                test(ra, T4, False, 'A')
            if R1:
                test(rb, T4, False, 'B')
        w4 += 448
        w6 += 64
        if w4 >= T4 and w6 >= T6:
            break
    res = []
    best = list(W.best)
    for fam in (0, 1):
        fa = info.fam[fam]
        ew = ENT6 if fam else ENT4
        for i in range(fa.n_resid):
            e = fa.off_resid + i * ew
            RA, RB = [int(x) for x in blob[e:e + 3]], [int(x) for x in blob[e + 3:e + 6]]
            ri = RA[2] >> IDX_SHIFT
            want = [(is6[l] if fam else is4[l]) and ri < (best[l] >> 32) for l in range(64)]
            if not any(want):
                break
            for l in range(64):
                ok = want[l] and _miss(RA, RB, ks[l], kd[l], proto[l], ports[l]) == 0
                if fam and ok:
                    ok = _miss6([int(x) for x in blob[e + 6:e + 9]], [int(x) for x in blob[e + 9:e + 12]],
                                RB[2], sw[l], tw[l]) == 0
                if ok:
                    best[l] = ri << 32 | (RB[2] >> OUT_SHIFT)
    if where is not None:
        for o, at in loc.items():
            if best[o] == W.best[o]:
                where[base + o] = at
    for l in range(64):
        hit = best[l] != (1 << 64) - 1
        out = best[l] & M32 if hit else 0
        if hit and out == OUT_ESCAPE:
            off_cold = info.fam[1 if is6[l] else 0].off_rec
            out = int(blob[off_cold + (best[l] >> 32)])
        res.append(out)
    if trace is not None:
        trace.append(dict(base=base, T4=T4, T6=T6, passes=passes))
    return res


def info_dir8(info):
    return info.fam[0].dims[0].dir8


def info_dir16(info):
    return info.fam[0].dims[0].off_dir16 != 0 or info.fam[1].dims[0].off_dir16 != 0


def emulate_pipe(blob, info, ns, slots, n, seed=0, trace=None, batches=None, where=None):
    """Verdicts of every packet (or of the listed batches only: others 0),
    one scratch carried from batch to batch as one wave would."""
    F = slot_fields(slots, n)
    W = Scratch(np.random.default_rng(seed))
    out = np.zeros(n, np.uint32)
    nb = (n + 63) // 64
    for b in (range(nb) if batches is None else batches):
        v = walk_batch(blob, info, ns, F, 64 * b, n, W, trace, where)
        m = min(64, n - 64 * b)
        out[64 * b:64 * b + m] = v[:m]
    return out
