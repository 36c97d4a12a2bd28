"""The pipelined flat-LDS walk (`classify_flat_pipe`) restated lane by lane
on the CPU (tests/pipe_emu.py) over the blobs the compiler produces, against
the oracle (first match in rule order, /root/reference/packet/acl.go:522-565).

VERDICT round 5 item 1(b): the model covers the walk's passes, windows,
marks and deltas (in a scratch carried from batch to batch with stale
contents), second passes (> 7 IPv4 rounds or > 1 IPv6 round in a batch),
and the 6-, 7- and 8-slot tables — so a GPU disagreement can be told apart
from a defect of the walk itself (the NS = 7 finding)."""
import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import oracle, rules_oracle as ro

import pipe_emu
from test_index_compile import compile_table


def _check(text: str, slots: np.ndarray, n: int):
    rules = nffacl.L3Rules.parse_text(text)
    blob, info = compile_table(rules, nffacl.ALGO_HYBRID)
    assert info.algo == nffacl.ALGO_HYBRID
    assert info.off_params > 0 and info.fam[0].entry_dwords == pipe_emu.ENT4  # flat-LDS positional
    ns = max(info.fam[0].n_slots, info.fam[1].n_slots)
    a4, a6 = ro.parse_text_table(text.encode()).arrays()
    want = oracle.classify_slots(slots, 64, n, a4, a6)
    trace = []
    got = pipe_emu.emulate_pipe(blob, info, ns, slots, n, seed=7, trace=trace)
    np.testing.assert_array_equal(got, want)
    return ns, trace


@pytest.mark.parametrize("fine_slots,ns", [(None, 6), ("7", 7), ("15", 8)])
def test_pipe_walk_c5(monkeypatch, fine_slots, ns):
    """C5 (10 k rules) at the default 6 slots and with the fine grids on 3 / 4
    grid slots (NFFACL_TUNE_FINE_SLOTS=7 / 15: the NS = 7 / 8 tables)."""
    if fine_slots:
        monkeypatch.setenv("NFFACL_TUNE_FINE_SLOTS", fine_slots)
    g = synth.gen_rules(synth.SPECS["c5"], synth.RULE_SEEDS["c5"])
    n = (1 << 12) + 5
    slots = synth.gen_slots(g, n, 61)
    got_ns, trace = _check(g.text, slots, n)
    assert got_ns == ns
    assert sum(t["T6"] > 0 for t in trace) > 0.9 * len(trace)  # IPv6 rounds in nearly every batch


def _dense_rules():
    """Lists long enough for several passes: 24 IPv4 rules over 10.0.0.0/9
    and 12 IPv6 rules over 2001:db8::/32 (every packet inside is a candidate
    of each), behind a selective tail that keeps the table a flat-LDS one."""
    lines = []
    for i in range(24):
        lines.append(f"ANY 10.0.0.0/9 {('TCP', 'UDP')[i % 2]} ANY {1000 + 97 * i}:{1100 + 97 * i} {i + 1}")
    for i in range(12):
        lines.append(f"ANY 2001:db8::/32 {('TCP', 'UDP')[i % 2]} ANY {2000 + 53 * i}:{2400 + 53 * i} {40 + i}")
    rng = np.random.default_rng(3)
    for i in range(3000):
        a = int(rng.integers(0, 1 << 24))
        lines.append(f"172.{a >> 16 & 255}.{a >> 8 & 255}.0/24 10.{i % 128}.{a & 255}.0/24 TCP ANY {i % 60000}:{i % 60000 + 9} {i % 9 + 1}")
    return "\n".join(lines) + "\n"


def test_pipe_walk_second_passes():
    """Batches past 7 IPv4 rounds (448 candidates) and past one IPv6 round
    (64) take second and third passes; the model's verdicts still equal the
    oracle's, stale scratch and all."""
    text = _dense_rules()
    g = synth.firewall_rules(text)
    n = 1 << 11
    slots = synth.gen_slots(g, n, 5)
    _, trace = _check(text, slots, n)
    passes = [len(t["passes"]) for t in trace]
    assert max(passes) >= 2, passes
    assert any(t["T4"] > 448 for t in trace) and any(t["T6"] > 64 for t in trace)


def _quad_perm_b1(v):
    """DPP quad_perm [1,0,3,2] over 64 lanes: lane l reads lane l ^ 1."""
    return v[np.arange(64) ^ 1]


def test_pair_gather_exchange():
    """classify.hpp pair_offsets / pair_unpack (the pipelined walk's pair
    gathers), restated lane by lane: both lanes of a pair load 12-byte pieces
    of ONE entry per instruction (even: piece p, odd: piece p + 1; X for the
    even lane's candidate, Y for the odd lane's), then trade across the pair.
    Every lane must end with exactly the pieces two plain loads of its own
    entry would give — for 24-byte IPv4 and 48-byte IPv6 entries, and with
    past-the-stream lanes pointing at offset 0."""
    rng = np.random.default_rng(7)
    tab = rng.integers(0, 2**32, size=1 << 14, dtype=np.uint64).astype(np.uint32)
    tab8 = tab.view(np.uint8)
    odd = (np.arange(64) & 1).astype(bool)

    def ld3(off):  # per-lane dwordx3 at byte offsets
        return np.stack([tab8[o:o + 12].view(np.uint32) for o in off])

    for ent_bytes in (24, 48):
        for trial in range(20):
            n_ent = (len(tab8) - 64) // ent_bytes
            o = rng.integers(0, n_ent, size=64).astype(np.uint32) * ent_bytes
            o[rng.random(64) < 0.2] = 0  # lanes past the stream
            p = _quad_perm_b1(o)
            h = np.where(odd, 12, 0).astype(np.uint32)
            oe = np.where(odd, p, o) + h
            od = np.where(odd, o, p) + h
            for base in ((0, 24) if ent_bytes == 48 else (0,)):
                X, Y = ld3(oe + base), ld3(od + base)
                send = np.where(odd[:, None], X, Y)
                r = _quad_perm_b1(send)
                lo = np.where(odd[:, None], r, X)
                hi = np.where(odd[:, None], Y, r)
                np.testing.assert_array_equal(lo, ld3(o + base))
                np.testing.assert_array_equal(hi, ld3(o + base + 12))
