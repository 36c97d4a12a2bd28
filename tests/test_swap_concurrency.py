"""Rule hot-swap while other threads classify (-m gpu).

The reference swaps *L3Rules with an atomic pointer store every few seconds
while flow-function clones keep classifying (examples/tutorial/step08.go:33-44);
include/nffacl.h promises nffacl_engine_swap_rules may run concurrently with
classification.  Here one thread loops nffacl_classify_host over 4 M packets,
another loops nffacl_classify_device on its own stream, a third runs a
batcher, while the main thread swaps between two rule sets 12+ times.  Every
batch must equal the oracle's verdicts for one of the two rule sets (the one
active when the call acquired its table) — a batch that read a freed or
half-overwritten table would match neither — and nothing may fault.
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


def _set(seed):
    g = synth.gen_rules(synth.SPECS["c2"], seed)
    return g, nffacl.L3Rules.parse_text(g.text), ro.parse_text_table(g.text.encode()).arrays()


def test_swap_while_classifying(torch_cuda):
    torch = torch_cuda
    g1, r1, (a4, a6) = _set(synth.RULE_SEEDS["c2"])
    _, r2, (b4, b6) = _set(synth.RULE_SEEDS["c2"] + 1)
    n_host = 1 << 22
    slots = synth.gen_slots(g1, n_host, 77)
    want = [oracle.classify_slots(slots, 64, n_host, a4, a6, threads=16),
            oracle.classify_slots(slots, 64, n_host, b4, b6, threads=16)]
    assert (want[0] != want[1]).mean() > 0.3  # the two answers are far apart
    n_dev = 1 << 20
    d_slots = torch.from_numpy(slots[:n_dev * 64]).to("cuda")
    frames = [slots[i * 64:(i + 1) * 64] for i in range(4096)]
    pk = np.frombuffer(slots[:4096 * 64], np.uint8)
    ptrs = (pk.ctypes.data + np.arange(4096, dtype=np.uint64) * 64).astype(np.uint64)
    del frames

    eng = nffacl.Engine(r1)
    bat = nffacl.Batcher(eng, stride=64, max_batch=4096, max_delay_us=50)
    stop = threading.Event()
    errors, seen = [], {"host": [], "dev": [], "bat": []}

    def which(got, sl):
        for k in (0, 1):
            if np.array_equal(got, want[k][sl]):
                return k
        return -1

    def host_loop():
        try:
            while not stop.is_set():
                port, _ = eng.classify_host(slots, 64, n_host)
                seen["host"].append(which(port, slice(0, n_host)))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    def dev_loop():
        try:
            s = torch.cuda.Stream()
            port = torch.zeros(n_dev, dtype=torch.int32, device="cuda")
            while not stop.is_set():
                with torch.cuda.stream(s):
                    eng.classify_device(d_slots, 64, n_dev, port, None, s)
                    s.synchronize()
                seen["dev"].append(which(port.cpu().numpy().view(np.uint32), slice(0, n_dev)))
        except Exception as e:  # pragma: no cover
            errors.append(e)

    def bat_loop():
        try:
            while not stop.is_set():
                got = bat.classify(ptrs[:2048], None)
                seen["bat"].append(which(got, slice(0, 2048)))
        except Exception as e:  # pragma: no cover
            errors.append(e)

    threads = [threading.Thread(target=f) for f in (host_loop, dev_loop, bat_loop)]
    for t in threads:
        t.start()
    swaps = 0
    t0 = time.time()
    while swaps < 12 or min(len(v) for v in seen.values()) < 4:
        eng.swap_rules(r2 if swaps % 2 == 0 else r1)
        swaps += 1
        time.sleep(0.02)
        assert time.time() - t0 < 90, {k: len(v) for k, v in seen.items()}
    stop.set()
    for t in threads:
        t.join()
    bat.close()
    eng.close()
    assert not errors, errors
    assert swaps >= 12
    for name, ks in seen.items():
        assert -1 not in ks, (name, ks)  # every batch = one rule set's oracle answer
    both = set(seen["host"]) | set(seen["dev"]) | set(seen["bat"])
    assert both == {0, 1}, seen


def test_frames_last_short_frame_ends_buffer(torch_cuda):
    """a short last frame that ends exactly at the end of the frame
    buffer (nothing readable after it) classifies like the oracle; the
    kernels read only chunks that start inside a frame."""
    torch = torch_cuda
    g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
    rules = nffacl.L3Rules.parse_text(g.text)
    a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
    m = 1024
    full = synth.gen_slots(g, m, 5, stride=64).reshape(m, 64)
    lens = np.random.default_rng(1).integers(0, 65, m)
    lens[-1] = 20
    offs = np.zeros(m, np.int64)
    buf = bytearray()
    for i in range(m):
        while len(buf) % 16:
            buf.append(0)
        offs[i] = len(buf)
        buf += full[i, :lens[i]].tobytes()
    frames = np.frombuffer(bytes(buf), np.uint8)
    assert offs[-1] + lens[-1] == len(frames)  # the last frame ends the buffer
    desc = (offs.astype(np.uint64) << np.uint64(16)) | lens.astype(np.uint64)
    want = oracle.classify_frames(frames, desc, a4, a6, threads=8)
    # the device buffer is exactly the frames: a 4 KiB-multiple allocation
    # holding them at its end
    pad = (-len(frames)) % 4096
    dev = torch.zeros(pad + len(frames), dtype=torch.uint8, device="cuda")
    dev[pad:] = torch.from_numpy(frames.copy()).to("cuda")
    d_desc = torch.from_numpy((desc + (np.uint64(pad) << np.uint64(16))).view(np.int64)).to("cuda")
    for algo in (nffacl.ALGO_LINEAR, nffacl.ALGO_INDEXED, nffacl.ALGO_HYBRID):
        with nffacl.Engine(rules, algo=algo) as eng:
            port = torch.zeros(m, dtype=torch.int32, device="cuda")
            eng.classify_frames_device(dev, d_desc, m, port)
            torch.cuda.synchronize()
        np.testing.assert_array_equal(port.cpu().numpy().view(np.uint32), want)


def test_bad_tuning_knob_rejected_at_creation(torch_cuda, monkeypatch):
    """Tuning knobs are read and validated once at engine creation."""
    rules = nffacl.L3Rules.parse_text(b"ANY ANY ANY ANY ANY Accept\n")
    for name, val in (("NFFACL_TUNE_BLOCK", "0"), ("NFFACL_TUNE_BLOCK", "100"), ("NFFACL_TUNE_ROUNDS", "3"),
                      ("NFFACL_TUNE_COAL", "x")):
        monkeypatch.setenv(name, val)
        with pytest.raises(nffacl.NFError):
            nffacl.Engine(rules)
        monkeypatch.delenv(name)
    with nffacl.Engine(rules) as eng:
        assert eng.algo in (nffacl.ALGO_INDEXED, nffacl.ALGO_LINEAR)
