#!/usr/bin/env python3
"""Launch-to-launch determinism of a config's batch kernel at the bench size:
K launches of 2^24 packets (pulled batches and all), every launch's verdicts
equal to the first on all packets, and a 2^16 sample equal to the oracle.
usage: python tools/determinism_check.py [c5|c2] [K]  -> one JSON line"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "nff-go_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402
from oracle import oracle, rules_oracle as ro  # noqa: E402  (checker only)

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
k = int(sys.argv[2]) if len(sys.argv) > 2 else 10
n = 1 << 24
g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
slots = synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg])
d = torch.from_numpy(slots).to("cuda")
eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
ports = [torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(2)]
eng.classify_device(d, 64, n, ports[0])
torch.cuda.synchronize()
diffs = []
for i in range(k):
    eng.classify_device(d, 64, n, ports[1])
    torch.cuda.synchronize()
    diffs.append(int((ports[0] != ports[1]).sum().item()))
a4, a6 = ro.parse_text_table(g.text.encode()).arrays()
idx = np.sort(np.random.default_rng(3).choice(n, 1 << 16, replace=False))
want = oracle.classify_slots(slots.reshape(n, 64)[idx].reshape(-1), 64, len(idx), a4, a6, threads=16)
got = ports[0].cpu().numpy().view(np.uint32)[idx]
print(json.dumps({"config": cfg, "launches": k, "packets": n, "differing_vs_first": diffs,
                  "oracle_sample_mismatches": int((got != want).sum())}))
