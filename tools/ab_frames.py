#!/usr/bin/env python3
"""C3 (IMIX packed frames) in one process: the classify kernel next to
speed-of-light kernels with its access pattern (tools/sol.hip `frames`:
descriptor + first 64-byte line per packet, trivial compute), interleaved.
usage: python tools/ab_frames.py [rounds]"""
import ctypes
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "nff-go_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
lib_path = ROOT / "tools" / "libsol.so"
if not lib_path.exists():
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    str(ROOT / "tools" / "sol.hip"), "-o", str(lib_path)], check=True)
sol = ctypes.CDLL(str(lib_path))
sol.sol_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
n = 1 << 24
g = synth.gen_rules(synth.SPECS["c3"], synth.RULE_SEEDS["c3"])
frames, desc = synth.gen_imix(g, n, synth.PACKET_SEEDS["c3"])
d_frames = torch.from_numpy(frames).to("cuda")
d_desc = torch.from_numpy(desc.view(np.int64)).to("cuda")
port = torch.empty(n, dtype=torch.int32, device="cuda")
bits = torch.empty(n // 64, dtype=torch.int64, device="cuda")
stream = torch.cuda.current_stream()
eng = nffacl.Engine(nffacl.L3Rules.parse_text(g.text))
V = {
    "classify": lambda: eng.classify_frames_device(d_frames, d_desc, n, port, bits, stream),
    "sol_frames": lambda: sol.sol_run(5, d_frames.data_ptr(), n, port.data_ptr(), bits.data_ptr(), d_desc.data_ptr(),
                                      8, 256, stream.cuda_stream),
    "sol_frames_pf": lambda: sol.sol_run(6, d_frames.data_ptr(), n, port.data_ptr(), bits.data_ptr(),
                                         d_desc.data_ptr(), 8, 256, stream.cuda_stream),
    "sol_frames_rs": lambda: sol.sol_run(7, d_frames.data_ptr(), n, port.data_ptr(), bits.data_ptr(),
                                         d_desc.data_ptr(), 8, 256, stream.cuda_stream),
    "sol_frames_rs_nt": lambda: sol.sol_run(8, d_frames.data_ptr(), n, port.data_ptr(), bits.data_ptr(),
                                            d_desc.data_ptr(), 8, 256, stream.cuda_stream),
    "sol_frames_16w": lambda: sol.sol_run(5, d_frames.data_ptr(), n, port.data_ptr(), bits.data_ptr(),
                                          d_desc.data_ptr(), 1, 1024, stream.cuda_stream),
}
times = {k: [] for k in V}
for _ in range(rounds):
    for k, f in V.items():
        for _ in range(2):
            f()
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for a, b in evs:
            a.record(stream)
            f()
            b.record(stream)
        torch.cuda.synchronize()
        times[k] += [a.elapsed_time(b) for a, b in evs]
bytes_pp = 76
out = {k: {"median_ms": float(np.median(v)), "Mpps": n / float(np.median(v)) / 1e3,
           "algorithmic_GBps": n * bytes_pp / float(np.median(v)) / 1e6} for k, v in times.items()}
print(json.dumps({"config": "c3", "packets": n, "mean_frame_stride_bytes": float(frames.nbytes / n),
                  "variants": out}, indent=1))
