#!/usr/bin/env python3
"""Batch kernel time while the resident consumer is armed (ADVICE round 3,
low: the consumer's workgroups hold LDS on their CUs for up to 100 ms).
Times the C2 and C5 device-resident batch (2^24 packets, HIP events) alone,
then with a scalar and a burst service kept hot by caller threads (C2 rules,
one call in flight per thread), then alone again.
usage: python tools/svc_overlap.py [threads]  -> one JSON line"""
import json
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "nff-go_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402

threads = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n = 1 << 24
stream = torch.cuda.current_stream()
port = torch.empty(n, dtype=torch.int32, device="cuda")
bits = torch.empty(n // 64, dtype=torch.int64, device="cuda")
work = {}
for cfg in ("c2", "c5"):
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
    slots = torch.from_numpy(synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg])).to("cuda")
    work[cfg] = (eng, slots)


def time_batch(cfg, reps=20):
    eng, slots = work[cfg]
    eng.classify_device(slots, 64, n, port, bits, stream)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(stream)
        eng.classify_device(slots, 64, n, port, bits, stream)
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in evs]))


g2 = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
rules2 = nffacl.L3Rules.parse_text(g2.text)
pk = synth.gen_slots(g2, 4096, synth.PACKET_SEEDS["c2"] + 5, stride=80)
out = {"threads_per_service": threads, "alone_ms": {c: time_batch(c) for c in work}}
scalar = nffacl.Service(0, mailboxes=64)
burst = nffacl.Service(0, mailboxes=32, burst=True)
stop = threading.Event()
calls = [0]


def caller(svc, is_burst, k):
    idx = [(k * 97 + i) % 4096 for i in range(32)]
    ptrs = np.array([pk.ctypes.data + 80 * i for i in idx], np.uint64)
    lens = np.full(32, 80, np.uint32)
    one = pk[80 * idx[0]:80 * idx[0] + 80]
    while not stop.is_set():
        if is_burst:
            svc.classify_burst(rules2, ptrs, lens)
        else:
            svc.classify(rules2, one)
        calls[0] += 1


ths = [threading.Thread(target=caller, args=(s, b, k)) for k in range(threads) for s, b in ((scalar, False), (burst, True))]
for t in ths:
    t.start()
time.sleep(0.3)
out["armed_ms"] = {c: time_batch(c) for c in work}
stop.set()
for t in ths:
    t.join()
out["calls_during"] = calls[0]
out["svc_stats"] = {"scalar": scalar.stats(), "burst": burst.stats()}
scalar.close()
burst.close()
time.sleep(0.3)
out["after_ms"] = {c: time_batch(c) for c in work}
out["slowdown_armed"] = {c: round(out["armed_ms"][c] / out["alone_ms"][c], 3) for c in work}
print(json.dumps(out))
