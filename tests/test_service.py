"""The scalar-call path (-m gpu): nffacl_service_* — one packet per call, the
rule set passed per call, answered by the persistent GPU consumer.

Reference call shape: pkt.L3ACLPermit(rules) / pkt.L3ACLPort(rules) inside a
SetSeparator / SetSplitter function (flow/flow.go:128, 1795-1797;
examples/firewall/firewall.go:54-57; examples/tutorial/step08.go:33-35).
Every verdict is checked against the oracle (or the reference's own known
answers); nothing here runs a CPU path of the product.
"""
import json
import threading
import time

import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import oracle, rules_oracle as ro

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.init()
    return torch


@pytest.fixture(scope="module")
def svc(torch_cuda):
    s = nffacl.Service(0, mailboxes=128, idle_us=2000)
    yield s
    s.close()


def _oracle_ports(text, frames, flags=0):
    a4, a6 = ro.parse_text_table(text.encode()).arrays()
    slots = np.zeros((len(frames), 80), np.uint8)
    for i, f in enumerate(frames):
        f = f[:80]
        slots[i, :len(f)] = np.frombuffer(f, np.uint8)
    return oracle.classify_slots(slots.reshape(-1), 80, len(frames), a4, a6, threads=8, flags=flags)


def test_match_kats(svc, golden):
    """All 7369 cases of acl_internal_test.go:501-1141: a one-rule L3Rules
    literal per case, one call each — the reference test's own shape."""
    z = np.load(golden / "acl_match_kats.npz", allow_pickle=False)
    pk = json.loads((golden / "kat_packets.json").read_text())
    frames = {name: bytes.fromhex(pk[name]) for name in z["packet_names"]}
    names = list(z["packet_names"])
    bad = []
    for fam in (4, 6):
        rules, want, pkt = z[f"c{fam}_rule"], z[f"c{fam}_want"], z[f"c{fam}_packet"]
        for i in range(len(rules)):
            rs = nffacl.L3Rules.from_arrays(rules[i:i + 1], None) if fam == 4 else \
                nffacl.L3Rules.from_arrays(None, rules[i:i + 1])
            got = svc.classify(rs, frames[names[int(pkt[i])]])
            if got != int(want[i]):
                bad.append((fam, i, got, int(want[i])))
    assert not bad, bad[:10]


def _c1(golden):
    """C1: the reference's examples/firewall/firewall.conf, packets drawn from C2's generator."""
    text = (golden / "rules" / "firewall.conf").read_text()
    return text, synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])


@pytest.mark.parametrize("cfg,n", [("c1", 4096), ("c2", 8192), ("c3", 4096), ("c5", 2048)])
def test_synthetic_vs_oracle(svc, golden, cfg, n):
    """C1 (firewall.conf), C2 (INDEXED), C3/C5 (HYBRID flat-LDS layout walked
    from global memory): per-packet calls == the oracle, ragged lengths too."""
    if cfg == "c1":
        text, g = _c1(golden)
    else:
        g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
        text = g.text
    rules = nffacl.L3Rules.parse_text(text)
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS["c2" if cfg == "c1" else cfg] + 11, stride=80).reshape(n, 80)
    rng = np.random.default_rng(5)
    lens = np.where(rng.random(n) < 0.2, rng.integers(0, 80, n), 80)
    frames = [bytes(slots[i, :lens[i]]) for i in range(n)]
    want = _oracle_ports(text, frames)
    got = np.array([svc.classify(rules, f) for f in frames], np.uint32)
    np.testing.assert_array_equal(got, want)


def test_linear_table(svc):
    """A rule set only LINEAR can encode (id_mask 0x0f, from_arrays only)."""
    r = np.zeros(3, nffacl.RULE4)
    r["output_number"] = [5, 6, 7]
    r["id"] = [0x06, 0x01, 0x00]
    r["id_mask"] = [0x0f, 0x0f, 0x00]
    rules = nffacl.L3Rules.from_arrays(r)
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    slots = synth.gen_slots(g, 512, 3, stride=80).reshape(512, 80)
    frames = [bytes(s) for s in slots]
    a4 = r.copy()
    want = oracle.classify_slots(slots.reshape(-1), 80, 512, a4, np.zeros(0, nffacl.RULE6), threads=4)
    got = np.array([svc.classify(rules, f) for f in frames], np.uint32)
    np.testing.assert_array_equal(got, want)


def test_vlan_flag(svc, golden):
    """ParseAllKnownL3CheckVLAN (vlan.go:104-117) per call: the tagged frame of
    vlan_test.go:23 hits an exact rule only with the flag."""
    kat = json.loads((golden / "vlan_kat.json").read_text())
    frame = bytes.fromhex(kat["hex"])
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules = nffacl.L3Rules.parse_text(g.text)
    frames = [frame, frame[:60], frame + b"\0" * 20]
    for flags in (0, nffacl.PARSE_VLAN):
        want = _oracle_ports(g.text, frames, flags)
        got = [svc.classify(rules, f, flags) for f in frames]
        assert got == [int(x) for x in want], (flags, got, want)


def test_threads_two_rule_sets(svc):
    """16 threads, each call naming one of two rule sets (alternating): every
    answer is the oracle's for the rule set of that call."""
    ga = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    gb = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"] + 1)
    ra, rb = nffacl.L3Rules.parse_text(ga.text), nffacl.L3Rules.parse_text(gb.text)
    n = 4096
    slots = synth.gen_slots(ga, n, 99, stride=80).reshape(n, 80)
    frames = [bytes(s) for s in slots]
    want = [_oracle_ports(ga.text, frames), _oracle_ports(gb.text, frames)]
    assert (want[0] != want[1]).mean() > 0.2
    errors = []

    def worker(t):
        try:
            for i in range(t, n, 16):
                which = (i // 16 + t) % 2
                got = svc.classify(ra if which == 0 else rb, frames[i])
                if got != want[which][i]:
                    errors.append((t, i, which, got, int(want[which][i])))
        except Exception as e:  # surfaced below
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errors, errors[:10]


@pytest.mark.parametrize("sleep_ns", ["-1", "0", "1500"])
def test_callers_nap_or_spin(torch_cuda, monkeypatch, sleep_ns):
    """More callers than mailboxes' waves and than a small CPU budget: callers
    that nap after posting (adaptive, or fixed) or spin — every answer the
    oracle's, no timeouts, the consumer never left its table."""
    monkeypatch.setenv("NFFACL_TUNE_SVC_SLEEP_NS", sleep_ns)
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules = nffacl.L3Rules.parse_text(g.text)
    n = 3000
    slots = synth.gen_slots(g, n, 5, stride=80).reshape(n, 80)
    frames = [bytes(s) for s in slots]
    want = _oracle_ports(g.text, frames)
    errors = []
    threads = 24

    with nffacl.Service(0, mailboxes=64) as s:
        def worker(t):
            try:
                for i in range(t, n, threads):
                    got = s.classify(rules, frames[i])
                    if got != want[i]:
                        errors.append((t, i, got, int(want[i])))
            except Exception as e:  # surfaced below
                errors.append(e)

        ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        st = s.stats()
    assert not errors, errors[:10]
    assert st["timeouts"] == 0 and st["table_oob"] == 0 and st["requests"] == n, st


def test_idle_exit_and_rearm(torch_cuda, golden):
    """The consumer leaves after idle_us without calls and the next call
    re-arms it; destroying a service whose consumer is resident returns
    promptly and leaves nothing running."""
    text, g = _c1(golden)
    rules = nffacl.L3Rules.parse_text(text)
    frame = bytes(synth.gen_slots(g, 1, 1, stride=80))
    want = int(_oracle_ports(text, [frame])[0])
    s = nffacl.Service(0, mailboxes=64, idle_us=500)
    assert s.classify(rules, frame) == want
    time.sleep(0.05)
    st = s.stats()
    assert st["running"] == 0 and st["launches"] == 1, st
    assert s.classify(rules, frame) == want
    assert s.stats()["launches"] == 2
    # busy: calls keep the consumer resident; destroy it mid-stream
    for _ in range(100):
        assert s.classify(rules, frame) == want
    assert s.stats()["running"] == 1
    t0 = time.perf_counter()
    s.close()
    assert time.perf_counter() - t0 < 0.5
    # a fresh service on the same device works after that
    with nffacl.Service(0, mailboxes=64) as s2:
        assert s2.classify(rules, frame) == want
    torch_cuda.cuda.synchronize()  # nothing left resident to wait for


def test_invalid_arguments(svc, golden):
    rules = nffacl.L3Rules.parse_text(_c1(golden)[0])
    with pytest.raises(nffacl.NFError):
        svc.classify(rules, b"\0" * 64, flags=2)
    with pytest.raises(nffacl.NFError):
        nffacl.Service(0, mailboxes=100)
    assert svc.classify(rules, b"") == 0  # empty frame: not IP


def test_no_table_walk_left_its_table(svc):
    """The consumer's bounds checks never fired over this module's calls."""
    st = svc.stats()
    assert st["table_oob"] == 0 and st["timeouts"] == 0, st
