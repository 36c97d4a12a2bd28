#!/usr/bin/env python3
"""Where C3's time goes: the same 2^24 IMIX frames classified, in one process,
against the C3 rule set, a 1-rule set (table walk ~free; HYBRID lane form and
INDEXED/LDS), and the 1k-rule C2 set (INDEXED, table in LDS).
usage: python tools/c3_floor.py [rounds]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "nff-go_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n = 1 << 24
g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
frames, desc = synth.gen_imix(g, n, synth.PACKET_SEEDS["c3"])
d_frames = torch.from_numpy(frames).to("cuda")
d_desc = torch.from_numpy(desc.view(np.int64)).to("cuda")
port = torch.empty(n, dtype=torch.int32, device="cuda")
bits = torch.empty(n // 64, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream()
c2 = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"]).text
one = "10.0.0.0/8 ANY TCP ANY 80 1\n"
engines = {
    "c3_rules_auto": nffacl.Engine(nffacl.L3Rules.parse_text(g.text)),
    "one_rule_hybrid": nffacl.Engine(nffacl.L3Rules.parse_text(one), algo=nffacl.ALGO_HYBRID),
    "one_rule_indexed_lds": nffacl.Engine(nffacl.L3Rules.parse_text(one), algo=nffacl.ALGO_INDEXED),
    "c2_rules_indexed_lds": nffacl.Engine(nffacl.L3Rules.parse_text(c2)),
}
times = {k: [] for k in engines}
for _ in range(rounds):
    for k, eng in engines.items():
        f = lambda: eng.classify_frames_device(d_frames, d_desc, n, port, bits, stream)  # noqa: E731
        f()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in evs:
            a.record(stream)
            f()
            b.record(stream)
        torch.cuda.synchronize()
        times[k] += [a.elapsed_time(b) for a, b in evs]
print(json.dumps({"packets": n, "algo": {k: e.algo for k, e in engines.items()},
                  "median_ms": {k: float(np.median(v)) for k, v in times.items()}}, indent=1))
