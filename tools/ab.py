#!/usr/bin/env python3
"""Interleaved A/B timing of classify launch variants in one process
(cdna_hip_programming.md §5.4 rule 24), with a bit-exactness check between
variants.  Variants are NFFACL_TUNE_* environment settings read per launch.
usage: python tools/ab.py [config] [rounds] [variant set: load]"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nff-go_amd"))
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 10
VARIANT_SETS = {
    "load": {
        "rows": {"NFFACL_TUNE_COAL": "0"},
        "coal_nt": {"NFFACL_TUNE_COAL": "2"},
        "rowswap_nt": {"NFFACL_TUNE_COAL": "4"},
        # speed-of-light kernels of tools/sol.hip on the same buffer (no classify):
        "sol_coalesced_nt": {"SOL": "3"},
        "sol_rows": {"SOL": "1"},
    },
}
VARIANTS = VARIANT_SETS[sys.argv[3] if len(sys.argv) > 3 else "load"]
n = 1 << 24
if cfg == "c1":
    text = (ROOT / "tests/golden/rules/firewall.conf").read_text()
    g = synth.firewall_rules(text)
else:
    g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
    text = g.text
slots = torch.from_numpy(synth.gen_slots(g, n, synth.PACKET_SEEDS[cfg])).to("cuda")
rules = nffacl.L3Rules.parse_text(text)
port = torch.empty(n, dtype=torch.int32, device="cuda")
bits = torch.empty(n // 64, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream()
eng = nffacl.Engine(rules)


_sol = None


def sol_lib():
    global _sol
    if _sol is None:
        import ctypes
        import subprocess
        lib_path = ROOT / "tools" / "libsol.so"
        if not lib_path.exists():
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                            str(ROOT / "tools" / "sol.hip"), "-o", str(lib_path)], check=True)
        _sol = ctypes.CDLL(str(lib_path))
        _sol.sol_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return _sol


def run(env, reps=10):
    if "SOL" in env:
        which = int(env["SOL"])
        per_cu, block = (4, 256) if which == 3 else (8, 256)
        launch = lambda: sol_lib().sol_run(which, slots.data_ptr(), n, port.data_ptr(), bits.data_ptr(),  # noqa: E731
                                           None, per_cu, block, stream.cuda_stream)
    else:
        launch = lambda: eng.classify_device(slots, 64, n, port, bits, stream)  # noqa: E731
    saved = {k: os.environ.get(k) for k in env if k != "SOL"}
    os.environ.update({k: v for k, v in env.items() if k != "SOL"})
    try:
        for _ in range(2):
            launch()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in evs:
            a.record(stream)
            launch()
            b.record(stream)
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in evs], port.clone(), bits.clone()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


times = {k: [] for k in VARIANTS}
ref = None
for r in range(rounds):
    for name, env in VARIANTS.items():
        ts, p, b = run(env)
        times[name] += ts
        if "SOL" in env:
            continue
        if ref is None:
            ref = (p, b)
        else:
            assert torch.equal(p, ref[0]) and torch.equal(b, ref[1]), f"variant {name} differs"
out = {k: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)), "Mpps": n / float(np.median(v)) / 1e3}
       for k, v in times.items()}
print(json.dumps({"config": cfg, "packets": n, "variants": out, "bit_identical": True}, indent=1))
