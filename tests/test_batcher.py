"""nffacl_batcher — many threads' bursts aggregated into shared GPU batches
(the reference's per-burst VectorSeparateFunction,
flow/flow.go:131, 1487-1520).  Every verdict comes from the HIP kernel; the
oracle checks each burst."""
import threading

import numpy as np
import pytest

import nffacl
from nffacl import synth
from oracle import oracle, rules_oracle as ro


def test_batcher_requires_engine():
    with pytest.raises(Exception):
        nffacl.Batcher(None)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch


@pytest.fixture(scope="module")
def workload():
    g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
    a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
    n = 1 << 16
    slots = synth.gen_slots(g, n, 0xBA7C, stride=80)
    want = oracle.classify_slots(slots, 80, n, a4, a6, threads=8)
    return g, slots, want


@pytest.mark.gpu
@pytest.mark.parametrize("threads,burst,delay", [(1, 32, 50), (8, 32, 100), (16, 7, 20), (4, 32, 0)])
def test_concurrent_bursts_bit_exact(torch_cuda, workload, threads, burst, delay):
    g, slots, want = workload
    n = len(want)
    lens = np.full(n, 80, np.uint32)
    lens[::5] = 64 + np.arange(len(lens[::5])) % 17  # ragged frame lengths
    # bytes past a frame's length must read as 0: compute the oracle on the clipped slots
    clipped = slots.reshape(n, 80).copy()
    for i in range(0, n, 5):
        clipped[i, lens[i]:] = 0
    a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
    want = oracle.classify_slots(clipped.reshape(-1), 80, n, a4, a6, threads=8)
    ptrs, lens = nffacl.Batcher.frame_pointers(slots, np.arange(n, dtype=np.uint64) * 80, lens)
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    got = np.zeros(n, np.uint32)
    errors = []
    with nffacl.Batcher(eng, stride=80, max_batch=4096, max_delay_us=delay, nbuf=3) as b:
        def worker(t):
            try:
                for s in range(t * burst, n, threads * burst):
                    e = min(n, s + burst)
                    got[s:e] = b.classify(ptrs[s:e], lens[s:e])
            except Exception as ex:  # surfaced below
                errors.append(ex)
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        st = b.stats()
    assert not errors, errors
    np.testing.assert_array_equal(got, want)
    assert st["packets"] == n and st["bursts"] == (n + burst - 1) // burst
    eng.close()


@pytest.mark.gpu
def test_submit_then_wait_and_flush(torch_cuda, workload):
    g, slots, want = workload
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    ptrs, lens = nffacl.Batcher.frame_pointers(slots, np.arange(len(want), dtype=np.uint64) * 80,
                                                np.full(len(want), 80, np.uint32))
    with nffacl.Batcher(eng, stride=80, max_batch=1024, max_delay_us=10_000_000, nbuf=4) as b:
        # three bursts queued before anyone waits; a huge delay means only flush ships them
        ts = [b.submit(ptrs[i * 32:(i + 1) * 32], lens[i * 32:(i + 1) * 32]) for i in range(3)]
        b.flush()
        for i, t in enumerate(ts):
            np.testing.assert_array_equal(b.wait(t), want[i * 32:(i + 1) * 32])
        # more than one batch worth of bursts from one thread, waited in order
        ts = [b.submit(ptrs[i * 32:(i + 1) * 32], lens[i * 32:(i + 1) * 32]) for i in range(3, 3 + 64)]
        b.flush()
        for i, t in zip(range(3, 3 + 64), ts):
            np.testing.assert_array_equal(b.wait(t), want[i * 32:(i + 1) * 32])
        # empty burst
        assert len(b.classify(ptrs[:0], lens[:0])) == 0
        with pytest.raises(nffacl.NFError):
            b.classify(ptrs[:2048], lens[:2048])  # > max_batch
    eng.close()


# ---- robustness (per-batch status, bounded waits, wait order) -------------------

def _c2_ptrs(workload):
    g, slots, want = workload
    ptrs, lens = nffacl.Batcher.frame_pointers(slots, np.arange(len(want), dtype=np.uint64) * 80,
                                                np.full(len(want), 80, np.uint32))
    return g, ptrs, lens, want


@pytest.mark.gpu
def test_failed_launch_fails_only_its_batch(torch_cuda, workload, monkeypatch):
    """One injected launch failure (NFFACL_TUNE_BATCH_FAIL_AT, read at
    creation): that burst gets the error, every later burst is served and
    bit-exact (no sticky error)."""
    g, ptrs, lens, want = _c2_ptrs(workload)
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    monkeypatch.setenv("NFFACL_TUNE_BATCH_FAIL_AT", "2")
    b = nffacl.Batcher(eng, stride=80, max_batch=1024, max_delay_us=50, nbuf=3)
    monkeypatch.delenv("NFFACL_TUNE_BATCH_FAIL_AT")
    try:
        np.testing.assert_array_equal(b.classify(ptrs[:32], lens[:32]), want[:32])
        with pytest.raises(nffacl.NFError) as ei:
            b.classify(ptrs[32:64], lens[32:64])
        assert ei.value.status == nffacl.ERR_HIP
        for k in range(2, 40):
            s = slice(32 * k, 32 * (k + 1))
            np.testing.assert_array_equal(b.classify(ptrs[s], lens[s]), want[s])
    finally:
        b.close()
        eng.close()


@pytest.mark.gpu
def test_wait_timeout_then_wait_again(torch_cuda, workload, monkeypatch):
    """A batch held back (NFFACL_TUNE_BATCH_HOLD: nothing ships before flush)
    never completes on its own: the bounded wait returns ERR_TIMEOUT and the
    ticket stays valid; after flush the same ticket yields the verdicts."""
    g, ptrs, lens, want = _c2_ptrs(workload)
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    monkeypatch.setenv("NFFACL_TUNE_BATCH_HOLD", "1")
    b = nffacl.Batcher(eng, stride=80, max_batch=1024, max_delay_us=10, nbuf=3)
    monkeypatch.delenv("NFFACL_TUNE_BATCH_HOLD")
    try:
        t = b.submit(ptrs[:32], lens[:32])
        with pytest.raises(nffacl.NFError) as ei:
            b.wait(t, timeout_us=3000)
        assert ei.value.status == nffacl.ERR_TIMEOUT
        b.flush()
        np.testing.assert_array_equal(b.wait(t, timeout_us=2_000_000), want[:32])
        with pytest.raises(nffacl.NFError) as ei:  # a second wait on the same ticket is rejected
            b.wait(t, timeout_us=1000)
        assert ei.value.status == nffacl.ERR_INVALID_ARG
    finally:
        b.close()
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nbuf", [2, 3, 4])
def test_partial_batches_ship_without_flush(torch_cuda, workload, nbuf):
    """A lone partial batch ships by itself at any nbuf (no flush), and a
    thread that queues bursts over several buffers may wait on its LAST
    ticket first (bounded waits: a regression fails instead of hanging)."""
    g, ptrs, lens, want = _c2_ptrs(workload)
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    try:
        with nffacl.Batcher(eng, stride=80, max_batch=64, max_delay_us=200, nbuf=nbuf) as b:
            t = b.submit(ptrs[:5], lens[:5])
            np.testing.assert_array_equal(b.wait(t, timeout_us=2_000_000), want[:5])
            k = nbuf - 1  # bursts filling nbuf - 1 buffers (each 64 = max_batch)
            ts = [b.submit(ptrs[64 * i:64 * (i + 1)], lens[64 * i:64 * (i + 1)]) for i in range(k)]
            ts.append(b.submit(ptrs[64 * k:64 * k + 7], lens[64 * k:64 * k + 7]))
            np.testing.assert_array_equal(b.wait(ts[-1], timeout_us=2_000_000), want[64 * k:64 * k + 7])
            for i in range(k):
                np.testing.assert_array_equal(b.wait(ts[i], timeout_us=2_000_000), want[64 * i:64 * (i + 1)])
    finally:
        eng.close()


@pytest.mark.gpu
def test_device_batcher_rules_per_burst(torch_cuda, workload):
    """A device batcher (no engine): 8 threads' bursts name one of two rule
    sets each; bursts of different rule sets never share a batch, and every
    burst equals the oracle for its own rule set."""
    g, slots, _ = workload
    gb = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"] + 7)
    texts = [g.text, gb.text]
    rs = [nffacl.L3Rules.parse_text(t) for t in texts]
    n = len(slots) // 80
    wants = []
    for t in texts:
        a4, a6 = ro.parse_text_table(t.encode()).arrays()
        wants.append(oracle.classify_slots(slots, 80, n, a4, a6, threads=8))
    assert (wants[0] != wants[1]).mean() > 0.2
    ptrs, lens = nffacl.Batcher.frame_pointers(slots, np.arange(n, dtype=np.uint64) * 80, np.full(n, 80, np.uint32))
    with pytest.raises(nffacl.NFError):  # a device batcher needs the rule set per burst
        with nffacl.Batcher(None, stride=80, device=0) as b0:
            b0.classify(ptrs[:4], lens[:4])
    errors = []
    with nffacl.Batcher(None, stride=80, max_batch=4096, max_delay_us=50, nbuf=4, device=0) as b:
        def worker(t):
            try:
                for s in range(t * 32, 16384, 8 * 32):
                    which = (s // 32 + t) % 2
                    got = b.classify(ptrs[s:s + 32], lens[s:s + 32], rules=rs[which])
                    if not np.array_equal(got, wants[which][s:s + 32]):
                        errors.append((t, s, which))
            except Exception as ex:
                errors.append(ex)
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        st = b.stats()
    assert not errors, errors[:5]
    assert st["bursts"] == 16384 // 32 and st["batches"] < st["bursts"]


@pytest.mark.gpu
def test_unwaited_tickets_bound_submit(torch_cuda, workload, monkeypatch):
    """One thread submits nbuf + 1 bursts spaced past max_delay without
    waiting: each burst ships alone and its uncollected ticket keeps its
    buffer busy, so the (nbuf + 1)-th submit cannot get a buffer from anyone
    but the caller itself.  It returns ERR_TIMEOUT after the bounded wait
    (NFFACL_TUNE_BATCH_SUBMIT_MS) instead of blocking forever; once the
    caller collects its tickets, submits work again and every verdict is
    exact."""
    import time
    g, ptrs, lens, want = _c2_ptrs(workload)
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    nbuf = 3
    monkeypatch.setenv("NFFACL_TUNE_BATCH_SUBMIT_MS", "200")
    b = nffacl.Batcher(eng, stride=80, max_batch=1024, max_delay_us=100, nbuf=nbuf)
    monkeypatch.delenv("NFFACL_TUNE_BATCH_SUBMIT_MS")
    try:
        ts = []
        for i in range(nbuf):
            ts.append(b.submit(ptrs[32 * i:32 * (i + 1)], lens[32 * i:32 * (i + 1)]))
            time.sleep(0.002)  # > max_delay: the burst's batch ships by itself
        t0 = time.monotonic()
        with pytest.raises(nffacl.NFError) as ei:
            b.submit(ptrs[32 * nbuf:32 * (nbuf + 1)], lens[32 * nbuf:32 * (nbuf + 1)])
        assert ei.value.status == nffacl.ERR_TIMEOUT
        assert 0.15 < time.monotonic() - t0 < 5.0
        for i, t in enumerate(ts):
            np.testing.assert_array_equal(b.wait(t, timeout_us=2_000_000), want[32 * i:32 * (i + 1)])
        for i in range(nbuf, nbuf + 8):
            t = b.submit(ptrs[32 * i:32 * (i + 1)], lens[32 * i:32 * (i + 1)])
            np.testing.assert_array_equal(b.wait(t, timeout_us=2_000_000), want[32 * i:32 * (i + 1)])
    finally:
        b.close()
        eng.close()


@pytest.mark.gpu
def test_tickets_collected_on_another_thread(torch_cuda, workload, monkeypatch):
    """a ticket collected on another thread than its
    submit still counts down its SUBMITTER's outstanding tickets (the counter
    rides with the burst), so the submitter is not taken for the holder of
    buffers it no longer holds: thread A's bursts are collected by thread B;
    thread C then fills every buffer and collects only after 0.6 s; A's next
    submit waits for C's buffers under the foreign bound
    (NFFACL_TUNE_BATCH_FOREIGN_MS, 3 s here) instead of failing after its own
    200 ms bound, and every verdict is exact."""
    import threading
    import time
    g, ptrs, lens, want = _c2_ptrs(workload)
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    nbuf = 3
    monkeypatch.setenv("NFFACL_TUNE_BATCH_SUBMIT_MS", "200")
    monkeypatch.setenv("NFFACL_TUNE_BATCH_FOREIGN_MS", "3000")
    b = nffacl.Batcher(eng, stride=80, max_batch=1024, max_delay_us=100, nbuf=nbuf)
    monkeypatch.delenv("NFFACL_TUNE_BATCH_SUBMIT_MS")
    monkeypatch.delenv("NFFACL_TUNE_BATCH_FOREIGN_MS")
    burst = lambda i: (ptrs[32 * i:32 * (i + 1)], lens[32 * i:32 * (i + 1)])  # noqa: E731
    try:
        ts = []
        for i in range(nbuf):  # thread A (this one)
            ts.append(b.submit(*burst(i)))
            time.sleep(0.002)
        got = {}

        def collect(tickets, first, delay=0.0):
            time.sleep(delay)
            for k, t in enumerate(tickets):
                got[first + k] = b.wait(t, timeout_us=2_000_000)
        tb = threading.Thread(target=collect, args=(ts, 0))  # thread B collects A's tickets
        tb.start()
        tb.join()
        tc_tickets = []

        def fill_then_collect():  # thread C
            for i in range(nbuf, 2 * nbuf):
                tc_tickets.append(b.submit(*burst(i)))
                time.sleep(0.002)
            collect(tc_tickets, nbuf, delay=0.6)
        tc = threading.Thread(target=fill_then_collect)
        tc.start()
        time.sleep(0.1)  # C holds every buffer now
        t0 = time.monotonic()
        t = b.submit(*burst(2 * nbuf))  # A: not its own tickets -> waits for C's
        waited = time.monotonic() - t0
        np.testing.assert_array_equal(b.wait(t, timeout_us=2_000_000), want[32 * 2 * nbuf:32 * (2 * nbuf + 1)])
        tc.join()
        assert waited > 0.3, waited
        for i in range(2 * nbuf):
            np.testing.assert_array_equal(got[i], want[32 * i:32 * (i + 1)])
    finally:
        b.close()
        eng.close()


@pytest.mark.gpu
def test_ticket_keeps_rules_alive(torch_cuda, workload):
    """A rule set made inline and dropped by the caller right after submit
    (b.submit(..., rules=L3Rules.parse_text(t))) stays alive until the
    ticket is waited for: the Ticket holds it (nffacl.h: rules must outlive
    the wait)."""
    import gc
    g, ptrs, lens, want = _c2_ptrs(workload)
    # (each burst names a rule set of its own, so each seals a batch: one buffer per burst)
    with nffacl.Batcher(None, stride=80, max_batch=1024, max_delay_us=20_000, nbuf=6, device=0) as b:
        ts = [b.submit(ptrs[32 * i:32 * (i + 1)], lens[32 * i:32 * (i + 1)], rules=nffacl.L3Rules.parse_text(g.text))
              for i in range(4)]
        gc.collect()
        for i, t in enumerate(ts):
            np.testing.assert_array_equal(b.wait(t, timeout_us=2_000_000), want[32 * i:32 * (i + 1)])
            assert t.rules is None
