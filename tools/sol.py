#!/usr/bin/env python3
"""Speed-of-light reference for the classify access pattern (tools/sol.hip),
next to the real classify kernel under launch-shape overrides.
usage: python tools/sol.py  (needs a GPU; builds tools/libsol.so if missing)"""
import ctypes
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "nff-go_amd"))
import torch  # noqa: E402

lib_path = ROOT / "tools" / "libsol.so"
if not lib_path.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(ROOT / "tools" / "sol.hip"), "-o", str(lib_path)], check=True)
lib = ctypes.CDLL(str(lib_path))
lib.sol_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

n = 1 << 24
slots = torch.randint(0, 255, (n * 64,), dtype=torch.uint8, device="cuda")
port = torch.empty(n, dtype=torch.int32, device="cuda")
bits = torch.empty(n // 64, dtype=torch.int64, device="cuda")
scratch = torch.empty(n * 64, dtype=torch.uint8, device="cuda")
stream = torch.cuda.current_stream()


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in evs)
    return ts[len(ts) // 2]


res = {}
names = {0: "rows_nt", 1: "rows", 2: "rows_prefetch_nt", 3: "coalesced_nt", 4: "copy_nt"}
for which, name in names.items():
    for per_cu, block in ((1, 1024), (2, 1024), (4, 256), (8, 256), (16, 256)):
        ms = timeit(lambda: lib.sol_run(which, slots.data_ptr(), n, port.data_ptr(), bits.data_ptr(),
                                        scratch.data_ptr(), per_cu, block, stream.cuda_stream))
        moved = n * 68 if which != 4 else n * 128
        res[f"{name} {per_cu}x{block}"] = {"ms": round(ms, 4), "GBps": round(moved / ms / 1e6, 1),
                                           "Mpps": round(n / ms / 1e3, 1)}
        print(name, per_cu, block, res[f"{name} {per_cu}x{block}"], flush=True)

# the real kernel under launch-shape overrides
import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402
g = synth.gen_rules(synth.SPECS["c2"], synth.RULE_SEEDS["c2"])
real = torch.from_numpy(synth.gen_slots(g, n, synth.PACKET_SEEDS["c2"])).to("cuda")
rules = nffacl.L3Rules.parse_text(g.text)
for per_cu, block in ((1, 1024), (2, 1024), (2, 512), (4, 256), (4, 512)):
    os.environ["NFFACL_TUNE_BLOCK"] = str(block)
    os.environ["NFFACL_TUNE_PER_CU"] = str(per_cu)
    with nffacl.Engine(rules) as eng:
        ms = timeit(lambda: eng.classify_device(real, 64, n, port, bits, stream))
    res[f"classify {per_cu}x{block}"] = {"ms": round(ms, 4), "Mpps": round(n / ms / 1e3, 1)}
    print("classify", per_cu, block, res[f"classify {per_cu}x{block}"], flush=True)
os.environ["NFFACL_TUNE_LDS"] = "0"
for per_cu, block in ((4, 256), (8, 256)):
    os.environ["NFFACL_TUNE_BLOCK"] = str(block)
    os.environ["NFFACL_TUNE_PER_CU"] = str(per_cu)
    with nffacl.Engine(rules) as eng:
        ms = timeit(lambda: eng.classify_device(real, 64, n, port, bits, stream))
    res[f"classify_global {per_cu}x{block}"] = {"ms": round(ms, 4), "Mpps": round(n / ms / 1e3, 1)}
    print("classify_global", per_cu, block, res[f"classify_global {per_cu}x{block}"], flush=True)
print(json.dumps(res))
