"""The burst call shape (-m gpu): nffacl_service_create_burst /
nffacl_service_classify_burst — a flow-function clone's whole burst (<= 32
packets) per call, the rule set named per call, answered by the resident
GPU consumer (one wave per mailbox), and the service failure policy.

Reference call shape: segmentProcess hands its VectorSeparateFunction one
burst at a time and waits for the answers (flow/flow.go:131, 1487-1520;
test/stability/testSingleWorkingFF.go:538-546).  Every verdict is checked
against the oracle; nothing here runs a CPU path of the product.
"""
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


def _want(text, slots, n, lens=None, flags=0):
    a4, a6 = ro.parse_text_table(text.encode()).arrays()
    s = slots.reshape(n, 80).copy()
    if lens is not None:
        for i in range(n):
            s[i, lens[i]:] = 0
    return oracle.classify_slots(s.reshape(-1), 80, n, a4, a6, threads=8, flags=flags)


def _ptrs(slots, n):
    return nffacl.Batcher.frame_pointers(slots, np.arange(n, dtype=np.uint64) * 80, np.full(n, 80, np.uint32))


@pytest.mark.parametrize("cfg,full_poll", [("c2", "1"), ("c3", "1"), ("c5", "1"), ("c2", "0"), ("c5", "0")])
def test_bursts_vs_oracle(torch_cuda, monkeypatch, cfg, full_poll):
    """C2 (INDEXED, LDS-staged), C3 / C5 (HYBRID flat, directories from
    global memory): bursts of 1..32 with ragged lengths == the oracle, with
    the consumer reading whole mailboxes every pass (default) or the header
    first and the packets on a new tag (NFFACL_TUNE_SVC_FULLPOLL=0)."""
    monkeypatch.setenv("NFFACL_TUNE_SVC_FULLPOLL", full_poll)
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    rules = nffacl.L3Rules.parse_text(g.text)
    n = 4096 if cfg != "c5" else 2048
    slots = synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg] + 21, stride=80)
    rng = np.random.default_rng(3)
    lens = np.where(rng.random(n) < 0.2, rng.integers(0, 80, n), 80).astype(np.uint32)
    want = _want(g.text, slots, n, lens)
    ptrs, _ = _ptrs(slots, n)
    got = np.zeros(n, np.uint32)
    with nffacl.Service(0, mailboxes=4, burst=True) as s:
        i = 0
        while i < n:
            k = min(n - i, int(rng.integers(1, 33)))
            got[i:i + k] = s.classify_burst(rules, ptrs[i:i + k], lens[i:i + k])
            i += k
        st = s.stats()
    np.testing.assert_array_equal(got, want)
    assert st["timeouts"] == 0 and st["table_oob"] == 0 and st["requests"] == n, st


def test_sixteen_clones_two_rule_sets_and_reload(torch_cuda):
    """16 clones x 32-packet bursts, each burst naming one of two rule sets,
    while a reloader swaps a third set in and out (step08.go:33-44: the rules
    pointer is read per call): every burst equals the oracle for the rule set
    it named."""
    texts = [synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"] + k).text for k in range(3)]
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    n = 16384
    slots = synth.gen_slots(g, n, 77, stride=80)
    wants = [_want(t, slots, n) for t in texts]
    assert (wants[0] != wants[1]).mean() > 0.2
    ptrs, lens = _ptrs(slots, n)
    current = [nffacl.L3Rules.parse_text(texts[0]), 0]
    errors = []
    stop = threading.Event()

    def reloader():
        k = 0
        while not stop.is_set():
            k ^= 2
            current[:] = [nffacl.L3Rules.parse_text(texts[k]), k]  # a new table every time
            time.sleep(0.002)

    with nffacl.Service(0, mailboxes=16, burst=True) as s:
        def clone(t):
            try:
                for b in range(t, n // 32, 16):
                    sl = slice(32 * b, 32 * b + 32)
                    if b % 2:
                        rs, which = current  # one read of the shared pointer per burst
                    else:
                        rs, which = fixed[1], 1
                    got = s.classify_burst(rs, ptrs[sl], lens[sl])
                    if not np.array_equal(got, wants[which][sl]):
                        errors.append((t, b, which))
            except Exception as e:  # surfaced below
                errors.append(e)

        fixed = [None, nffacl.L3Rules.parse_text(texts[1])]
        rl = threading.Thread(target=reloader)
        rl.start()
        ths = [threading.Thread(target=clone, args=(t,)) for t in range(16)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        stop.set()
        rl.join()
        st = s.stats()
    assert not errors, errors[:5]
    assert st["timeouts"] == 0 and st["table_oob"] == 0, st


def test_scalar_call_on_burst_service_and_vlan(torch_cuda, golden):
    """A one-packet call on a burst service is a burst of one; the VLAN flag
    applies to the whole burst (vlan_test.go:23's tagged frame)."""
    import json
    kat = json.loads((golden / "vlan_kat.json").read_text())
    frame = np.frombuffer(bytes.fromhex(kat["hex"])[:80].ljust(80, b"\0"), np.uint8)
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    rules = nffacl.L3Rules.parse_text(g.text)
    slots = np.tile(frame, 32).copy()
    ptrs, lens = _ptrs(slots, 32)
    with nffacl.Service(0, mailboxes=2, burst=True) as s:
        for flags in (0, nffacl.PARSE_VLAN):
            want = _want(g.text, slots, 32, flags=flags)
            np.testing.assert_array_equal(s.classify_burst(rules, ptrs, lens, flags=flags), want)
            assert s.classify(rules, bytes(frame), flags) == want[0]
        with pytest.raises(nffacl.NFError):  # > 32 packets
            s.classify_burst(rules, np.tile(ptrs, 2), np.tile(lens, 2))
        assert len(s.classify_burst(rules, ptrs[:0], lens[:0])) == 0
        # lengths given as int64 / a list are converted
        # into an array that stays alive for the call (not a freed temporary)
        want = _want(g.text, slots, 32)
        for ln in (lens.astype(np.int64), [int(x) for x in lens]):
            np.testing.assert_array_equal(s.classify_burst(rules, ptrs, ln), want)
        with pytest.raises(ValueError):
            s.classify_burst(rules, ptrs, lens[:5])


@pytest.mark.parametrize("burst", [False, True])
def test_stalled_consumer_policy(torch_cuda, monkeypatch, burst):
    """Failure policy (nffacl.h): with the consumer stopped (pause) a call
    re-posts once, then withdraws its request and returns ERR_TIMEOUT with
    verdict 0 within 2 x the timeout; the reference-shaped L3ACLPort returns
    0 without raising; the rules may be freed at once (the withdrawn request
    is answered without a table read); after resume every call is exact
    again and no table walk left its table."""
    import gc
    monkeypatch.setenv("NFFACL_TUNE_SVC_TIMEOUT_US", "20000")
    s = nffacl.Service(0, mailboxes=64 if not burst else 4, burst=burst)
    monkeypatch.delenv("NFFACL_TUNE_SVC_TIMEOUT_US")
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    n = 64
    slots = synth.gen_slots(g, n, 9, stride=80)
    want = _want(g.text, slots, n)
    ptrs, lens = _ptrs(slots, n)
    frames = [bytes(slots[80 * i:80 * i + 80]) for i in range(n)]
    try:
        rules = nffacl.L3Rules.parse_text(g.text)
        assert s.classify(rules, frames[0]) == want[0]
        s.pause(True)
        t0 = time.monotonic()
        with pytest.raises(nffacl.NFError) as ei:
            if burst:
                s.classify_burst(rules, ptrs[:32], lens[:32])
            else:
                s.classify(rules, frames[1])
        dt = time.monotonic() - t0
        assert ei.value.status == nffacl.ERR_TIMEOUT
        assert 0.03 < dt < 1.0, dt
        assert s.L3ACLPort(rules, frames[2]) == 0  # the policy's verdict, no exception
        if burst:
            assert (s.L3ACLPortBurst(rules, ptrs[:8], lens[:8]) == 0).all()
        st = s.stats()
        assert st["timeouts"] == (3 if burst else 2) and st["retries"] == st["timeouts"], st
        del rules  # freed right after the timeouts: the withdrawn requests name no table
        gc.collect()
        s.pause(False)
        rules = nffacl.L3Rules.parse_text(g.text)
        for i in range(0, n, 32):
            if burst:
                np.testing.assert_array_equal(s.classify_burst(rules, ptrs[i:i + 32], lens[i:i + 32]), want[i:i + 32])
            for k in range(i, i + 8):
                assert s.classify(rules, frames[k]) == want[k]
        st = s.stats()
        assert st["table_oob"] == 0 and st["timeouts"] == (3 if burst else 2), st
    finally:
        s.close()
