#!/usr/bin/env python3
"""Interleaved A/B of NFFACL_TUNE_* launch variants on one workload in one
process, with verdicts compared bit for bit against the first variant.
usage: python tools/ab_env.py CONFIG ROUNDS NAME=VAR:VAL[,VAR:VAL] ...
CONFIG: c2 | c5 (64-byte slots) | c3 (IMIX frames) | l2 (L2 ACL, 256 rules)."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "nff-go_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402

cfg, rounds = sys.argv[1], int(sys.argv[2])
variants = {}
for spec in sys.argv[3:]:
    name, _, kv = spec.partition("=")
    variants[name] = dict(x.split(":") for x in kv.split(",") if x)
n = 1 << 24
# one engine per variant, compiled under the variant's environment (table
# layout knobs such as NFFACL_TUNE_FLAT act at compile time, launch knobs at
# every launch)
if cfg == "l2":
    g = synth.gen_l2_rules(256)
    make = lambda: nffacl.L2Engine(nffacl.L2Rules.parse_text(g.text))  # noqa: E731
else:
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    make = lambda: nffacl.Engine(nffacl.L3Rules.parse_text(g.text))  # noqa: E731
engines = {}
port = torch.empty(n, dtype=torch.int32, device="cuda")
bits = torch.empty(n // 64, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream()
if cfg == "c3":
    frames, desc = synth.gen_imix(g, n, synth.PACKET_SEEDS[cfg])
    d_frames = torch.from_numpy(frames).to("cuda")
    d_desc = torch.from_numpy(desc.view(np.int64)).to("cuda")
    run = lambda eng: eng.classify_frames_device(d_frames, d_desc, n, port, bits, stream)  # noqa: E731
elif cfg == "l2":
    slots = torch.from_numpy(synth.gen_l2_slots(g, n)).to("cuda")
    run = lambda eng: eng.classify_device(slots, 64, n, port, bits, stream)  # noqa: E731
else:
    slots = torch.from_numpy(synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg])).to("cuda")
    run = lambda eng: eng.classify_device(slots, 64, n, port, bits, stream)  # noqa: E731


def with_env(env, f):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return f()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


print(f"{cfg}: inputs ready", file=sys.stderr, flush=True)  # (progress: a silent GPU run reads as hung)
ref = None
exact = {}
for name, env in variants.items():
    engines[name] = with_env(env, make)
    with_env(env, lambda: run(engines[name]))
    torch.cuda.synchronize()
    got = port.cpu().numpy().copy()
    if ref is None:
        ref = got
    exact[name] = bool((got == ref).all())
    print(f"{name}: bit-exact {exact[name]}", file=sys.stderr, flush=True)
times = {k: [] for k in variants}
for _ in range(rounds):
    for name, env in variants.items():
        def timed():
            eng = engines[name]
            run(eng)
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for a, b in evs:
                a.record(stream)
                run(eng)
                b.record(stream)
            torch.cuda.synchronize()
            return [a.elapsed_time(b) for a, b in evs]
        times[name] += with_env(env, timed)
    print(f"round {_}: " + " ".join(f"{k} {np.median(v):.4f}" for k, v in times.items()), file=sys.stderr, flush=True)
out = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)), "Gpps": n / float(np.median(v)) / 1e6,
           "bit_exact_vs_first": exact[k]} for k, v in times.items()}
print(json.dumps({"config": cfg, "packets": n, "rounds": rounds, "variants": out,
                  "env": variants}, indent=1))
