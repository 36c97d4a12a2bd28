#!/usr/bin/env python3
"""Host-inclusive classify (nffacl_classify_host) variants on one GPU: the
kernel reading pinned slots over PCIe (zero-copy) vs DMA'd chunks, buffers in
flight, chunk size; verdicts into a pinned array (written by the kernels over
PCIe) or a pageable one (copied out).  Every variant is checked bit for bit
against the device-resident classify of the same packets.
usage: python tools/host_modes.py [CONFIG] [PACKETS_LOG2]"""
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / "nff-go_amd"), str(ROOT)]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nffacl  # noqa: E402
from nffacl import synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
m = 1 << (int(sys.argv[2]) if len(sys.argv) > 2 else 23)
g = synth.gen_rules(synth.SPECS[cfg], synth.RULE_SEEDS[cfg])
rules = nffacl.L3Rules.parse_text(g.text)
slots = synth.gen_slots(g, m, synth.PACKET_SEEDS[cfg])
pinned = torch.from_numpy(slots).pin_memory()
pin_np = pinned.numpy()
out_pin = torch.empty(m, dtype=torch.int32).pin_memory().numpy().view(np.uint32)
ref_eng = nffacl.Engine(rules)
d_slots = torch.from_numpy(slots).to("cuda")
ref = torch.empty(m, dtype=torch.int32, device="cuda")
ref_eng.classify_device(d_slots, 64, m, ref, None, torch.cuda.current_stream())
torch.cuda.synchronize()
ref = ref.cpu().numpy().view(np.uint32)
del d_slots

variants = [("zc_b2_c20", {"NFFACL_TUNE_HOST_DMA": "0", "NFFACL_TUNE_HOST_BUFS": "2", "NFFACL_TUNE_HOST_CHUNK": "20"}),
            ("zc_b3_c20", {"NFFACL_TUNE_HOST_DMA": "0", "NFFACL_TUNE_HOST_BUFS": "3", "NFFACL_TUNE_HOST_CHUNK": "20"}),
            ("zc_b2_c22", {"NFFACL_TUNE_HOST_DMA": "0", "NFFACL_TUNE_HOST_BUFS": "2", "NFFACL_TUNE_HOST_CHUNK": "22"}),
            ("zc_b4_c18", {"NFFACL_TUNE_HOST_DMA": "0", "NFFACL_TUNE_HOST_BUFS": "4", "NFFACL_TUNE_HOST_CHUNK": "18"}),
            ("dma_b2_c20", {"NFFACL_TUNE_HOST_DMA": "1", "NFFACL_TUNE_HOST_BUFS": "2", "NFFACL_TUNE_HOST_CHUNK": "20"}),
            ("dma_b3_c20", {"NFFACL_TUNE_HOST_DMA": "1", "NFFACL_TUNE_HOST_BUFS": "3", "NFFACL_TUNE_HOST_CHUNK": "20"}),
            ("dma_b4_c20", {"NFFACL_TUNE_HOST_DMA": "1", "NFFACL_TUNE_HOST_BUFS": "4", "NFFACL_TUNE_HOST_CHUNK": "20"}),
            ("dma_b4_c18", {"NFFACL_TUNE_HOST_DMA": "1", "NFFACL_TUNE_HOST_BUFS": "4", "NFFACL_TUNE_HOST_CHUNK": "18"})]
res = {}
for name, env in variants:
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    eng = nffacl.Engine(rules)
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    r = {}
    for oname, out in (("pinned_out", out_pin), ("pageable_out", None)):
        eng.classify_host(pin_np, 64, m, out=out, permit=False)  # warm-up (buffers)
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            port, _ = eng.classify_host(pin_np, 64, m, out=out, permit=False)
            ts.append(time.perf_counter() - t)
        r[oname] = {"mpps": round(m / min(ts) / 1e6, 1), "ms": round(min(ts) * 1e3, 3),
                    "gbps_in": round(m * 64 / min(ts) / 1e9, 1), "bit_exact": bool((port[:m] == ref).all())}
    eng.close()
    res[name] = r
    print(name, r, file=sys.stderr, flush=True)
print(json.dumps({"config": cfg, "packets": m, "variants": res}))
