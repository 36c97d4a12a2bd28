"""The INDEXED table compiler (host C++) checked on CPU: a numpy model of the
kernel's lookup (radix bucket -> ordered candidate list ->
full rule test, min over key dimensions + residual scan) run over the blob
nffacl_table_compile() produces must give the oracle's first match on every
packet.  This validates the compiled structure without a device; the HIP
kernel walking the same blob is checked against the oracle in
test_gpu_parity.py."""
import ctypes

import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import oracle, rules_oracle as ro


class DimInfo(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint32), ("shift", ctypes.c_uint32), ("n_buckets", ctypes.c_uint32),
                ("off_dir", ctypes.c_uint32), ("off_cands", ctypes.c_uint32), ("n_rules", ctypes.c_uint32),
                ("max_list", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("n_cands", ctypes.c_uint64)]


class FamInfo(ctypes.Structure):
    _fields_ = [("n_dims", ctypes.c_uint32), ("off_rec", ctypes.c_uint32), ("n_rec", ctypes.c_uint32),
                ("off_resid", ctypes.c_uint32), ("n_resid", ctypes.c_uint32), ("dims", DimInfo * 4)]


class TableInfo(ctypes.Structure):
    _fields_ = [("algo", ctypes.c_int32), ("reserved", ctypes.c_uint32), ("blob_dwords", ctypes.c_uint64),
                ("fam", FamInfo * 2)]


def compile_table(rules: nffacl.L3Rules, algo=nffacl.ALGO_INDEXED):
    f = nffacl._lib.nffacl_table_compile
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(TableInfo)]
    info = TableInfo()
    assert f(rules.handle, algo, None, 0, ctypes.byref(info)) == 0
    blob = np.zeros(info.blob_dwords, np.uint32)
    assert f(rules.handle, algo, blob.ctypes.data, len(blob), ctypes.byref(info)) == 0
    return blob, info


def bswap(x):
    x = x.astype(np.uint32)
    return ((x & 0xFF) << 24) | ((x & 0xFF00) << 8) | ((x >> 8) & 0xFF00) | (x >> 24)


def fields(slots: np.ndarray, n: int):
    """Header fields of 64-byte slots with IHL 5 / IPv6 (test traffic only)."""
    p = slots.reshape(n, 64).astype(np.uint32)
    le = lambda o: p[:, o] | p[:, o + 1] << 8 | p[:, o + 2] << 16 | p[:, o + 3] << 24  # noqa: E731
    et = p[:, 12] << 8 | p[:, 13]
    is4, is6 = et == 0x0800, et == 0x86DD
    ihl5 = (p[:, 14] & 0xF) == 5
    s = np.stack([np.where(is6, le(22 + 4 * k), le(26) if k == 0 else 0) for k in range(4)])
    t = np.stack([np.where(is6, le(38 + 4 * k), le(30) if k == 0 else 0) for k in range(4)])
    proto = np.where(is6, p[:, 20], p[:, 23])
    po = np.where(is6, 54, 34)
    rows = np.arange(n)
    sp = p[rows, po] << 8 | p[rows, po + 1]
    dp = p[rows, po + 2] << 8 | p[rows, po + 3]
    return dict(is4=is4 & ihl5, is6=is6, s=s, t=t, proto=proto, sp=sp, dp=dp, skip=is4 & ~ihl5)


def match(blob, off_rec, v6, r, F, sel):
    """Full rule test of record r[i] against packet sel[i] (vectorised)."""
    rw = 20 if v6 else 8
    rec = blob[off_rec + r[:, None] * rw + np.arange(rw)[None, :]]
    m = np.zeros(len(r), np.uint32)
    if v6:
        for k in range(4):
            m |= (F["s"][k][sel] ^ rec[:, k]) & rec[:, 4 + k]
            m |= (F["t"][k][sel] ^ rec[:, 8 + k]) & rec[:, 12 + k]
        meta, lo, hi, out = rec[:, 16], rec[:, 17], rec[:, 18], rec[:, 19]
    else:
        m |= (F["s"][0][sel] ^ rec[:, 0]) & rec[:, 1]
        m |= (F["t"][0][sel] ^ rec[:, 2]) & rec[:, 3]
        meta, lo, hi, out = rec[:, 4], rec[:, 5], rec[:, 6], rec[:, 7]
    m |= (F["proto"][sel] ^ meta) & ((meta >> 8) & 0xFF)
    sp, dp = F["sp"][sel], F["dp"][sel]
    ok = (m == 0) & (sp >= (lo & 0xFFFF)) & (sp <= (hi & 0xFFFF)) & (dp >= (lo >> 16)) & (dp <= (hi >> 16))
    return ok, out


def emulate(blob, info, F, n):
    best = np.full(n, 0xFFFFFFFF, np.uint64)
    outv = np.zeros(n, np.uint32)
    for fam, v6 in ((0, False), (1, True)):
        fi = info.fam[fam]
        mine = F["is6"] if v6 else F["is4"]
        for d in range(fi.n_dims):
            di = fi.dims[d]
            kind = di.kind
            key = {0: bswap(F["s"][0]), 1: bswap(F["t"][0]), 2: bswap(F["s"][0]), 3: bswap(F["t"][0]),
                   4: F["sp"], 5: F["dp"]}[kind].astype(np.uint64)
            dirv = blob[di.off_dir:di.off_dir + di.n_buckets + 1].astype(np.int64)
            t = (key >> np.uint64(di.shift)).astype(np.int64)
            assert (t < di.n_buckets).all()
            start, end = dirv[t], dirv[t + 1]
            for k in range(di.max_list):
                live = mine & (start + k < end)
                if not live.any():
                    break
                sel = np.nonzero(live)[0]
                r = blob[di.off_cands + start[sel] + k].astype(np.uint64)
                keep = r < best[sel]
                sel, r = sel[keep], r[keep]
                ok, out = match(blob, fi.off_rec, v6, r.astype(np.int64), F, sel)
                best[sel[ok]] = r[ok]
                outv[sel[ok]] = out[ok]
                start[sel[ok]] = end[sel[ok]]  # stop scanning this list
        for i in range(fi.n_resid):
            r = int(blob[fi.off_resid + i])
            sel = np.nonzero(mine & (best > r))[0]
            ok, out = match(blob, fi.off_rec, v6, np.full(len(sel), r), F, sel)
            best[sel[ok]] = r
            outv[sel[ok]] = out[ok]
    return best, outv


def check(text: str, slots: np.ndarray, n: int):
    rules = nffacl.L3Rules.parse_text(text)
    blob, info = compile_table(rules)
    assert info.algo == nffacl.ALGO_INDEXED
    a4, a6 = ro.parse_text_table(text.encode()).arrays()
    want, which = oracle.classify_slots_which(slots, 64, n, a4, a6)
    F = fields(slots, n)
    best, out = emulate(blob, info, F, n)
    sel = ~F["skip"]
    got = np.where(best != 0xFFFFFFFF, out, 0)
    np.testing.assert_array_equal(got[sel], want[sel])
    # every bucket list ascends (first-match order is preserved)
    for fam in range(2):
        fi = info.fam[fam]
        for d in range(fi.n_dims):
            di = fi.dims[d]
            dirv = blob[di.off_dir:di.off_dir + di.n_buckets + 1].astype(np.int64)
            assert dirv[0] == 0 and dirv[-1] == di.n_cands and (np.diff(dirv) >= 0).all()
            c = blob[di.off_cands:di.off_cands + int(di.n_cands)].astype(np.int64)
            first = np.zeros(len(c), bool)
            first[dirv[:-1][dirv[:-1] < len(c)]] = True
            assert (np.diff(c)[~first[1:]] > 0).all()
    return info


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_index_matches_oracle_synthetic(cfg):
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    n = 1 << 15
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg])
    info = check(g.text, slots, n)
    fi = info.fam[0]
    assert fi.n_dims >= 2 and fi.n_resid < 10


def test_index_firewall(golden):
    text = (golden / "rules" / "firewall.conf").read_text()
    g = synth.firewall_rules(text)
    n = 1 << 14
    check(text, synth.gen_slots(g, n, 5), n)


def test_index_nested_and_overlapping_rules():
    """Heavily nested prefixes, duplicates, port ranges and residual rules."""
    lines = []
    rng = np.random.default_rng(9)
    for i in range(600):
        plen = int(rng.integers(0, 33))
        a = int(rng.integers(0, 1 << 32)) & (0xFFFFFFFF << (32 - plen) if plen else 0) & 0xFFFFFFFF
        a = (a & 0x0FFFFFFF) | 0x0A000000 if plen >= 8 else a  # cluster inside 10/8
        src = f"{a >> 24}.{a >> 16 & 255}.{a >> 8 & 255}.{a & 255}/{plen}" if i % 5 else "ANY"
        dst = "ANY" if i % 3 else f"10.{i % 256}.0.0/16"
        proto = ["ANY", "TCP", "UDP"][i % 3]
        lo = int(rng.integers(0, 60000))
        dp = "ANY" if i % 4 else f"{lo}:{lo + int(rng.integers(0, 5000))}"
        lines.append(f"{src} {dst} {proto} ANY {dp} {i % 7}")
    lines.append("ANY ANY TCP ANY ANY 9")  # residual catch-all for TCP
    text = "\n".join(lines) + "\n"
    g = synth.firewall_rules(text)
    n = 1 << 14
    check(text, synth.gen_slots(g, n, 6), n)


def test_linear_table_has_no_index():
    rules = nffacl.L3Rules.parse_text(b"10.0.0.0/8 ANY ANY ANY ANY 1\n")
    _, info = compile_table(rules, nffacl.ALGO_LINEAR)
    assert info.algo == nffacl.ALGO_LINEAR and info.fam[0].n_dims == 0
