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
