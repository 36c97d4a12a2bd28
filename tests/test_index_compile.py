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
                ("off_dir", ctypes.c_uint32), ("off_entries", ctypes.c_uint32), ("n_rules", ctypes.c_uint32),
                ("max_list", ctypes.c_uint32), ("off_dir16", ctypes.c_uint32), ("n_entries", ctypes.c_uint64),
                ("kind2", ctypes.c_uint32), ("shift2", ctypes.c_uint32), ("bits2", ctypes.c_uint32),
                ("dir8", ctypes.c_uint32)]


MAX_SLOTS = 8
KIND_NONE = 6


class FamInfo(ctypes.Structure):
    _fields_ = [("n_rec", ctypes.c_uint32), ("off_rec", ctypes.c_uint32), ("entry_dwords", ctypes.c_uint32),
                ("off_resid", ctypes.c_uint32), ("n_resid", ctypes.c_uint32), ("dims", DimInfo * MAX_SLOTS),
                ("n_slots", ctypes.c_uint32), ("off_ent_base", ctypes.c_uint32)]


class TableInfo(ctypes.Structure):
    _fields_ = [("algo", ctypes.c_int32), ("lds_dwords", ctypes.c_uint32), ("blob_dwords", ctypes.c_uint64),
                ("fam", FamInfo * 2), ("off_params", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


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


def match(blob, offs, v6, F, sel):
    """Full rule test of the entries at dword offsets offs[i] against packet
    sel[i] (vectorised); returns (ok, rule index, output number)."""
    ew = 20 if v6 else 8
    e = blob[offs[:, None] + np.arange(ew)[None, :]]
    m = (F["s"][0][sel] ^ e[:, 0]) & e[:, 1]
    m |= (F["t"][0][sel] ^ e[:, 2]) & e[:, 3]
    meta, lo, hi, out = e[:, 4], e[:, 5], e[:, 6], e[:, 7]
    if v6:  # extension: s1 s2 s3 sm1 sm2 sm3 t1 t2 t3 tm1 tm2 tm3
        for k in range(3):
            m |= (F["s"][k + 1][sel] ^ e[:, 8 + k]) & e[:, 11 + k]
            m |= (F["t"][k + 1][sel] ^ e[:, 14 + k]) & e[:, 17 + k]
    exact = (meta >> 8) & 1
    m |= np.where(exact == 1, (F["proto"][sel] ^ meta) & 0xFF, 0)
    sp, dp = F["sp"][sel], F["dp"][sel]
    ok = (m == 0) & (sp >= (lo & 0xFFFF)) & (sp <= (hi & 0xFFFF)) & (dp >= (lo >> 16)) & (dp <= (hi >> 16))
    return ok, (meta >> 9).astype(np.uint64), out


KEYS = {0: lambda F: bswap(F["s"][0]), 1: lambda F: bswap(F["t"][0]), 2: lambda F: bswap(F["s"][0]),
        3: lambda F: bswap(F["t"][0]), 4: lambda F: F["sp"], 5: lambda F: F["dp"]}


def bucket_of(di, F):
    """Bucket index of every packet in slot di: key >> shift, or for a 2-D
    slot (kind2 != none) (key >> shift) << bits2 | key2 >> shift2."""
    t = KEYS[di.kind](F).astype(np.uint64) >> np.uint64(di.shift)
    if di.kind2 != KIND_NONE:
        t = (t << np.uint64(di.bits2)) | (KEYS[di.kind2](F).astype(np.uint64) >> np.uint64(di.shift2))
    return t.astype(np.int64)


def dir_values(blob, di):
    """dir[0..n_buckets] of a slot: plain u32, or two-level (table.hpp:
    dir[t] = base[t >> 6] + u16 dir16[t], or base[t >> 4] + u8 dir8[t])."""
    nb = di.n_buckets
    if di.off_dir16 == 0:
        return blob[di.off_dir:di.off_dir + nb + 1].astype(np.int64)
    t = np.arange(nb + 1)
    if di.dir8 == 2:  # 4-bit counts per bucket, a base per 16 buckets (table.hpp kDir4GroupShift)
        tb = np.arange(nb)
        cnt = (blob[di.off_dir16 + (tb >> 3)].astype(np.int64) >> (4 * (tb & 7))) & 0xF
        out = np.zeros(nb + 1, np.int64)
        for g in range((nb + 15) // 16):
            seg = cnt[16 * g:16 * g + 16]
            out[16 * g:16 * g + len(seg) + 1] = int(blob[di.off_dir + g]) + np.concatenate([[0], np.cumsum(seg)])
        return out
    if di.dir8:
        base = blob[di.off_dir + (t >> 4)].astype(np.int64)
        w = blob[di.off_dir16 + (t >> 2)].astype(np.int64)
        return base + ((w >> (8 * (t & 3))) & 0xFF)
    base = blob[di.off_dir + (t >> 6)].astype(np.int64)
    w = blob[di.off_dir16 + (t >> 1)].astype(np.int64)
    rel = np.where(t & 1, w >> 16, w & 0xFFFF)
    return base + rel


def emulate(blob, info, F, n):
    best = np.full(n, 0xFFFFFFFF, np.uint64)
    outv = np.zeros(n, np.uint32)
    for fam, v6 in ((0, False), (1, True)):
        fi = info.fam[fam]
        ew = fi.entry_dwords
        mine = F["is6"] if v6 else F["is4"]
        for d in range(4):
            di = fi.dims[d]
            if di.n_rules == 0:
                continue
            key = KEYS[di.kind](F).astype(np.uint64)
            dirv = dir_values(blob, di)
            t = (key >> np.uint64(di.shift)).astype(np.int64)
            assert (t < di.n_buckets).all()
            start, end = dirv[t], dirv[t + 1]
            for k in range(di.max_list):
                live = mine & (start + k < end)
                if not live.any():
                    break
                sel = np.nonzero(live)[0]
                ok, idx, out = match(blob, di.off_entries + (start[sel] + k) * ew, v6, F, sel)
                keep = idx < best[sel]
                ok &= keep
                best[sel[ok]] = idx[ok]
                outv[sel[ok]] = out[ok]
                stop = ok | ~keep
                start[sel[stop]] = end[sel[stop]]  # hit, or list passed best
        for i in range(fi.n_resid):
            sel = np.nonzero(mine)[0]
            ok, idx, out = match(blob, np.full(len(sel), fi.off_resid + i * ew), v6, F, sel)
            ok &= idx < best[sel]
            best[sel[ok]] = idx[ok]
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
    # every bucket list ascends in rule index (first-match order is preserved)
    for fam in range(2):
        fi = info.fam[fam]
        ew = fi.entry_dwords
        for d in range(4):
            di = fi.dims[d]
            dirv = dir_values(blob, di)
            assert dirv[0] == 0 and dirv[-1] == di.n_entries and (np.diff(dirv) >= 0).all()
            c = blob[di.off_entries + 4 + ew * np.arange(int(di.n_entries))].astype(np.int64) >> 9
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
    assert fi.dims[0].n_rules > 0 and fi.dims[1].n_rules > 0 and fi.n_resid < 10


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
    assert info.algo == nffacl.ALGO_LINEAR and info.fam[0].entry_dwords == 0


def test_non_indexable_rules_compile_linear():
    """id_mask outside {0, 0xff} (only reachable through from_arrays) -> LINEAR."""
    r = np.zeros(1, nffacl.RULE4)
    r["id_mask"] = 0x0F
    _, info = compile_table(nffacl.L3Rules.from_arrays(r), nffacl.ALGO_INDEXED)
    assert info.algo == nffacl.ALGO_LINEAR


# ---- HYBRID (table.hpp "hybrid table") --------------------------------------

def pmask(L):
    """Top-L-bits mask of a big-endian word, L in 0..32."""
    L = L.astype(np.uint64)
    return ((np.uint64(0xFFFFFFFF00000000) >> L) & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def hyb_test(blob, info, offs, v6, F, sel):
    """Exact flat-form entries (table.hpp) at dword offsets offs[i] against
    packet sel[i]: addresses under their prefix lengths, protocol, ports;
    returns (ok, rule index, output code)."""
    ew = 12 if v6 else 6
    e = blob[offs[:, None] + np.arange(ew)[None, :]]
    lens = e[:, 5]
    sl, dl = (lens & 0xFF).astype(np.int64), ((lens >> 8) & 0xFF).astype(np.int64)
    m = np.zeros(len(sel), np.uint32)
    for k in range(4 if v6 else 1):
        rs = e[:, 0] if k == 0 else e[:, 5 + k]
        rd = e[:, 1] if k == 0 else e[:, 8 + k]
        m |= (bswap(F["s"][k][sel]) ^ rs) & pmask(np.clip(sl - 32 * k, 0, 32))
        m |= (bswap(F["t"][k][sel]) ^ rd) & pmask(np.clip(dl - 32 * k, 0, 32))
    meta = e[:, 2]
    m |= np.where((meta >> 8) & 1 == 1, (F["proto"][sel] ^ meta) & 0xFF, 0).astype(np.uint32)
    sp, dp = F["sp"][sel].astype(np.uint32), F["dp"][sel].astype(np.uint32)
    lo, hi = e[:, 3], e[:, 4]
    ok = (m == 0) & (sp >= (lo & 0xFFFF)) & (sp <= (hi & 0xFFFF)) & (dp >= (lo >> 16)) & (dp <= (hi >> 16))
    return ok, (meta >> 9).astype(np.uint64), (lens >> 16).astype(np.uint32)


def emulate_hybrid(blob, info, F, n):
    """Flat forms: every candidate of every list (no early exit), the minimum
    passing rule index wins; its output number from the entry's 16-bit code,
    or from the family's output array when the code is 0xFFFF."""
    best = np.full(n, 0xFFFFFFFF, np.uint64)
    code = np.zeros(n, np.uint32)

    def post(sel, ok, idx, out):
        better = ok & (idx < best[sel])
        best[sel[better]] = idx[better]
        code[sel[better]] = out[better]

    for fam, v6 in ((0, False), (1, True)):
        fi = info.fam[fam]
        ew = fi.entry_dwords
        assert ew == (12 if v6 else 6)
        mine = F["is6"] if v6 else F["is4"]
        for d in range(fi.n_slots):
            di = fi.dims[d]
            if di.n_rules == 0:
                continue
            dirv = dir_values(blob, di)  # global (flat) or LDS image (flat-LDS)
            t = bucket_of(di, F)
            assert (t < di.n_buckets).all()
            start, end = dirv[t], dirv[t + 1]
            for k in range(di.max_list):
                live = mine & (start + k < end)
                if not live.any():
                    break
                sel = np.nonzero(live)[0]
                offs = fi.off_ent_base + (start[sel] + k) * ew
                post(sel, *hyb_test(blob, info, offs, v6, F, sel))
        for i in range(fi.n_resid):
            sel = np.nonzero(mine)[0]
            offs = np.full(len(sel), fi.off_resid + ew * i)
            post(sel, *hyb_test(blob, info, offs, v6, F, sel))
    out = np.zeros(n, np.uint32)
    hit = best != 0xFFFFFFFF
    out[hit] = code[hit]
    for fam, v6 in ((0, False), (1, True)):
        rd = (F["is6"] if v6 else F["is4"]) & hit & (code == 0xFFFF)
        out[rd] = blob[info.fam[fam].off_rec + best[rd].astype(np.int64)]
    return best, out


def check_hybrid(text: str, slots: np.ndarray, n: int, dir_kb=None, monkeypatch=None):
    rules = nffacl.L3Rules.parse_text(text)
    if dir_kb is not None:
        monkeypatch.setenv("NFFACL_TUNE_DIR_KB", str(dir_kb))
    blob, info = compile_table(rules, nffacl.ALGO_HYBRID)
    assert info.algo == nffacl.ALGO_HYBRID
    a4, a6 = ro.parse_text_table(text.encode()).arrays()
    want, _ = oracle.classify_slots_which(slots, 64, n, a4, a6)
    F = fields(slots, n)
    # lane form (directories in LDS): INDEXED's inline entries; flat forms: exact 6/12-dword entries
    lane = info.fam[0].entry_dwords == 8
    best, out = emulate(blob, info, F, n) if lane else emulate_hybrid(blob, info, F, n)
    sel = ~F["skip"]
    got = np.where(best != 0xFFFFFFFF, out, 0)
    np.testing.assert_array_equal(got[sel], want[sel])
    return info


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_hybrid_matches_oracle_synthetic(cfg):
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    n = 1 << 15
    info = check_hybrid(g.text, synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg]), n)
    assert 0 < info.lds_dwords * 4 <= 128 * 1024  # LDS directories (flat-LDS form)
    assert info.fam[0].dims[0].off_dir16 != 0  # two-level (u16) directories


@pytest.mark.parametrize("flat", [0, 2])
def test_hybrid_lds_forms_u32_directories(monkeypatch, flat):
    """NFFACL_TUNE_DIR16=0: the lane form (0) and the flat-LDS form (2) with
    plain u32 LDS directories."""
    monkeypatch.setenv("NFFACL_TUNE_DIR16", "0")
    monkeypatch.setenv("NFFACL_TUNE_FLAT", str(flat))
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
    n = 1 << 14
    info = check_hybrid(g.text, synth.gen_slots(g, n, 41), n)
    assert info.lds_dwords > 0 and info.fam[0].dims[0].off_dir16 == 0
    assert (info.fam[0].entry_dwords == 6) == (flat == 2)


@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
def test_hybrid_lane_form(cfg, monkeypatch):
    """NFFACL_TUNE_FLAT=0: INDEXED's inline entries walked per lane over the
    LDS directories."""
    monkeypatch.setenv("NFFACL_TUNE_FLAT", "0")
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    n = 1 << 13
    info = check_hybrid(g.text, synth.gen_slots(g, n, 43), n)
    assert info.lds_dwords > 0 and info.fam[0].entry_dwords == 8


def test_hybrid_small_directory_budget(monkeypatch):
    """A 4 KiB directory budget forces long lists; still the first match."""
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
    n = 1 << 13
    info = check_hybrid(g.text, synth.gen_slots(g, n, 11), n, dir_kb=4, monkeypatch=monkeypatch)
    assert info.lds_dwords * 4 <= 4 * 1024 + 64


def test_hybrid_firewall_and_nested(golden):
    text = (golden / "rules" / "firewall.conf").read_text()
    n = 1 << 13
    check_hybrid(text, synth.gen_slots(synth.firewall_rules(text), n, 5), n)
    lines = []
    rng = np.random.default_rng(10)
    for i in range(400):
        plen = int(rng.integers(0, 33))
        a = int(rng.integers(0, 1 << 32)) & (0xFFFFFFFF << (32 - plen) if plen else 0) & 0xFFFFFFFF
        src = f"{a >> 24}.{a >> 16 & 255}.{a >> 8 & 255}.{a & 255}/{plen}" if i % 5 else "ANY"
        dst = "ANY" if i % 3 else f"10.{i % 256}.0.0/16"
        proto = ["ANY", "TCP", "UDP", "ICMP"][i % 4]
        lo = int(rng.integers(0, 60000))
        sp = "ANY" if i % 2 or proto == "ICMP" else f"{lo & ~8191}:{(lo & ~8191) + 8191}"  # whole blocks
        dp = "ANY" if i % 4 == 0 or proto == "ICMP" else f"{lo}:{lo + int(rng.integers(0, 5000))}"
        lines.append(f"{src} {dst} {proto} {sp} {dp} {i % 7}")
        if i % 50 == 0:
            lines.append(f"ANY 2001:db8:{i:x}::/{48 + i % 80} TCP ANY {lo} {i}")
    lines.append("ANY ANY UDP ANY ANY 9")
    text = "\n".join(lines) + "\n"
    check_hybrid(text, synth.gen_slots(synth.firewall_rules(text), n, 6), n)


@pytest.mark.parametrize("cfg", ["c2", "c3"])
def test_hybrid_flat_form_synthetic(cfg, monkeypatch):
    """Directories past LDS size force the flat form (compact entries + cold
    records) on the small configs too."""
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    n = 1 << 14
    info = check_hybrid(g.text, synth.gen_slots(g, n, 31), n, dir_kb=1024, monkeypatch=monkeypatch)
    assert info.lds_dwords == 0 and info.fam[0].entry_dwords == 6


def test_hybrid_falls_back_on_non_cidr_masks():
    r = np.zeros(1, nffacl.RULE4)
    r["src_mask"] = 0x00FF00FF  # not a prefix
    r["output_number"] = 1
    _, info = compile_table(nffacl.L3Rules.from_arrays(r), nffacl.ALGO_HYBRID)
    assert info.algo == nffacl.ALGO_INDEXED


def test_hybrid_policy_c5_flat(monkeypatch):
    """C5 (100k rules): the flat-LDS form (compact entries, LDS directories)
    and, with NFFACL_TUNE_FLAT=1, global directories with generalized 1-D /
    2-D slots (lds_dwords == 0).  Both give the oracle's first match."""
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    n = 1 << 12
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c5"])
    monkeypatch.setenv("NFFACL_TUNE_FLAT", "2")
    info = check_hybrid(g.text, slots, n)
    assert 0 < info.lds_dwords * 4 <= 135 * 1024 and info.fam[0].entry_dwords == 6
    assert info.fam[0].dims[3].n_rules == 0  # sparse source-port slot folded away
    assert info.fam[0].dims[0].dir8 == 2  # 4-bit-count two-level directories (round 5)
    monkeypatch.setenv("NFFACL_TUNE_DIR4", "0")
    info = check_hybrid(g.text, slots, n)
    assert info.fam[0].dims[0].dir8 == 1  # u8 two-level directories
    monkeypatch.delenv("NFFACL_TUNE_DIR4")
    monkeypatch.setenv("NFFACL_TUNE_FLAT", "1")
    info = check_hybrid(g.text, slots, n)
    assert info.lds_dwords == 0 and info.fam[0].entry_dwords == 6
    assert any(info.fam[0].dims[k].kind2 != KIND_NONE for k in range(info.fam[0].n_slots))  # 2-D slots


@pytest.mark.parametrize("cfg", ["c2", "c3", "c5"])
@pytest.mark.parametrize("flat,slots2d", [("1", "0"), ("1", "1"), ("2", "2")])
def test_hybrid_generalized_slots(cfg, flat, slots2d, monkeypatch):
    """Generalized slots (global directories, or LDS-budgeted two-level ones):
    every rule listed in every bucket of its 1-D or 2-D slot that its ranges
    meet; first match == oracle."""
    monkeypatch.setenv("NFFACL_TUNE_FLAT", flat)
    monkeypatch.setenv("NFFACL_TUNE_SLOTS2D", slots2d)
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    n = 1 << 13
    info = check_hybrid(g.text, synth.gen_slots(g, n, 61), n)
    for fam in info.fam:
        assert 1 <= fam.n_slots <= MAX_SLOTS
        for k in range(fam.n_slots):
            assert fam.dims[k].n_rules > 0


@pytest.mark.parametrize("cfg", ["c3", "c5"])
def test_hybrid_flat_lds_form(cfg, monkeypatch):
    """NFFACL_TUNE_FLAT=2: compact entries + cold records walked flat, with
    the directories (two-level, absolute entry numbers in the base words)
    as the LDS image."""
    monkeypatch.setenv("NFFACL_TUNE_FLAT", "2")
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    n = 1 << 13
    info = check_hybrid(g.text, synth.gen_slots(g, n, 51), n)
    assert 0 < info.lds_dwords * 4 <= 135 * 1024
    assert info.fam[0].entry_dwords == 6 and info.fam[0].dims[0].off_dir16 != 0


@pytest.mark.parametrize("flat", ["1", "2"])
def test_hybrid_large_output_numbers(flat, monkeypatch):
    """OutputNumbers past the entries' 16-bit code (65535 and up, to the u32
    maximum parseRuleResult accepts) come from the output arrays."""
    monkeypatch.setenv("NFFACL_TUNE_FLAT", flat)
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
    lines = g.text.splitlines()
    big = [65534, 65535, 65536, 70000, 4294967295]
    for i in range(1, len(lines)):
        if i % 3 == 0:
            f = lines[i].split()
            f[5] = str(big[i % len(big)])
            lines[i] = " ".join(f)
    text = "\n".join(lines) + "\n"
    n = 1 << 13
    check_hybrid(text, synth.gen_slots(synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"]), n, 71), n)


@pytest.mark.parametrize("coarse,dir8", [("1", "1"), ("1", "0"), ("0", "0")])
def test_hybrid_c5_coarse_slots_and_directory_forms(coarse, dir8, monkeypatch):
    """The flat-LDS layout knobs: coarse address slots for short prefixes on
    or off, u8 or u16 two-level directories; every combination gives the
    oracle's first match (the default, u8 without coarse slots, runs in
    test_hybrid_policy_c5_flat)."""
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    n = 1 << 12
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c5"])
    monkeypatch.setenv("NFFACL_TUNE_COARSE", coarse)
    monkeypatch.setenv("NFFACL_TUNE_DIR8", dir8)
    monkeypatch.setenv("NFFACL_TUNE_FINE_A", "0")  # the four 1-D slots only (fine grids: below)
    info = check_hybrid(g.text, slots, n)
    assert info.fam[0].dims[0].dir8 == int(dir8)
    kinds = [info.fam[0].dims[k].kind for k in range(info.fam[0].n_slots)]
    if coarse == "1":  # compacted slots: the sport slot dropped, src (0) and dst (1) twice
        assert 4 not in kinds and kinds.count(0) == 2 and kinds.count(1) == 2
    else:
        assert info.fam[0].n_slots == 4


def check_param_block(blob, info):
    """The flat-LDS slot parameter block (table.hpp kFlatParamDwords) holds
    each positional slot's shift, directory offsets and fine-grid bits for
    both families, and lies inside the staged LDS image."""
    assert info.off_params > 0 and info.off_params + 4 * MAX_SLOTS <= info.lds_dwords
    P = blob[info.off_params:info.off_params + 4 * MAX_SLOTS].reshape(MAX_SLOTS, 4)
    for f in range(2):
        fi = info.fam[f]
        for s in range(fi.n_slots):
            d = fi.dims[s]
            w = (P[s] >> np.uint32(16 * f)) & np.uint32(0xFFFF)
            assert int(w[0]) == d.shift and int(w[1]) == d.off_dir and int(w[2]) == d.off_dir16, (f, s)
            if s >= 4:
                assert int(w[3]) & 0xFF == d.bits2 and int(w[3]) >> 8 == d.shift2, (f, s)


@pytest.mark.parametrize("cfg,env", [
    ("c5", {}),
    ("c5", {"NFFACL_TUNE_FINE_A": "0"}),
    ("c5", {"NFFACL_TUNE_FINE_A": "8", "NFFACL_TUNE_FINE_P": "4", "NFFACL_TUNE_FINE_MIN": "16",
            "NFFACL_TUNE_FINE_SLOTS": "15"}),
    ("c5", {"NFFACL_TUNE_FINE_A": "8", "NFFACL_TUNE_FINE_P": "3", "NFFACL_TUNE_FINE_SLOTS": "3"}),
    ("c3", {"NFFACL_TUNE_FINE_A": "8", "NFFACL_TUNE_FINE_MIN": "16", "NFFACL_TUNE_DIR_PER_RULE": "16"}),
])
def test_hybrid_fine_slots_and_param_block(monkeypatch, cfg, env):
    """Fine 2-D address x port grids (positional slots 4..7) and the LDS
    parameter block: the emulated walk of the compiled blob equals the
    oracle, the grids are 2-D slots on (address, port), and the parameter
    block matches the slot table."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    n = 1 << 13
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg] + 3)
    info = check_hybrid(g.text, slots, n)
    rules = nffacl.L3Rules.parse_text(g.text)
    blob, info = compile_table(rules, nffacl.ALGO_HYBRID)
    check_param_block(blob, info)
    fine = [info.fam[0].dims[k] for k in range(4, info.fam[0].n_slots) if info.fam[0].dims[k].n_rules]
    if env.get("NFFACL_TUNE_FINE_A") == "0":
        assert not fine and info.fam[0].n_slots == 4
    else:  # default: 9 x 5 grids on slots 4-5 (dst x dport, src x dport)
        assert fine and all(d.kind2 != KIND_NONE for d in fine)
        if cfg == "c5" and not env:
            assert info.fam[0].n_slots == 6


def _c5_plus(extra_lines):
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    return g, g.text + "".join(line + "\n" for line in extra_lines)


@pytest.mark.parametrize("case", ["grid_overflow", "dir_overflow"])
def test_hybrid_fine_grids_when_offsets_overflow(case):
    """fine 2-D grids take their directory bytes off
    the LDS budget in the u8 form.  A grid whose lists overflow the u8
    offsets sheds the rules of its overflowing groups (they stay in their
    1-D slots), and when a 1-D slot overflows them the directories re-size
    for the wider form with the grids' bytes in that form taken off the
    budget: the image always fits kHybLdsDirMaxBytes and the walk still
    gives the oracle's first match.  grid_overflow: 300 rules (dst /9, dport
    8192-9000) that the dst x dport grid would put into one bucket;
    dir_overflow: 300 copies of one dst /32 rule (one 1-D bucket of 300
    entries).  Both end in the u16 form beside C5's own grids."""
    if case == "grid_overflow":
        extra = ["ANY 33.128.0.0/9 TCP ANY 8192:9000 Accept"] * 300
    else:
        extra = ["ANY 44.55.66.77/32 UDP 1000:2000 ANY Reject"] * 300
    g, text = _c5_plus(extra)
    n = 1 << 12
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c5"] + 11)
    # a few packets aimed at the added rules (IPv4 TCP, dst 33.200.1.2 / 44.55.66.77)
    for i in range(0, n, 97):
        pk = slots[i * 64:(i + 1) * 64]
        pk[12:14] = (0x08, 0x00)
        pk[14] = 0x45
        pk[23] = 6 if case == "grid_overflow" else 17
        pk[30:34] = (33, 200, 1, 2) if case == "grid_overflow" else (44, 55, 66, 77)
        pk[34:38] = (0x05, 0xDC, 0x21, 0x98)  # sport 1500, dport 8600
    info = check_hybrid(text, slots, n)
    assert info.lds_dwords * 4 <= 135 * 1024
    fine = [info.fam[0].dims[k] for k in range(4, info.fam[0].n_slots) if info.fam[0].dims[k].n_rules]
    assert fine and all(d.max_list < 300 for d in fine)  # the C5 rules' own grids stay, without the hot bucket
    assert info.fam[0].dims[0].dir8 == 0 and info.fam[0].dims[0].off_dir16 != 0  # u16 form


@pytest.mark.parametrize("env", [{"NFFACL_TUNE_FINE_A": "10"}, {"NFFACL_TUNE_FINE_A": "9", "NFFACL_TUNE_FINE_P": "7"}])
def test_hybrid_oversized_fine_grids_fall_back(monkeypatch, env):
    """Layout knobs whose fine 2-D grids would push the flat-LDS image past
    the staged-image limit (FINE_A = 10 at C5: 271 KB) compile without the
    grids instead (or, failing that, with global directories): the image
    always fits and the walk still gives the oracle's first match."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    n = 1 << 12
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c5"] + 13)
    info = check_hybrid(g.text, slots, n)
    assert info.lds_dwords * 4 <= 135 * 1024
