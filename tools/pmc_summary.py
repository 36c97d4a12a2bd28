#!/usr/bin/env python3
"""Summarise a tools/gpu_prof.sh run: mean per-dispatch counters of the
classify kernel + kernel-trace stats.  usage: pmc_summary.py <prof dir> [kernel substring]"""
import collections
import csv
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
key = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "k_indexed_slots"
out = {}
for sub in ("fetch", "write", "sq", "sq2", "tcc", "ta"):
    f = d / sub / "run_counter_collection.csv"
    if not f.exists():
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
stats = {}
f = d / "trace" / "run_kernel_stats.csv"
if f.exists():
    for r in csv.DictReader(open(f)):
        if key in r["Name"]:
            stats = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                     "max_ns": float(r["MaxNs"])}
res = {"kernel": key, "trace": stats, "counters_mean_per_dispatch": out}
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    res["hbm_bytes_per_launch"] = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
if out.get("TCC_HIT_sum") is not None and out.get("TCC_MISS_sum") is not None:
    res["l2_hit_rate"] = out["TCC_HIT_sum"] / max(1.0, out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
waves = out.get("SQ_WAVES")
if waves and "SQ_INSTS_VALU" in out:
    batches = None
    res["per_wave"] = {k: out[k] / waves for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD") if k in out}
print(json.dumps(res, indent=1))
# --traffic-key cfg:algo:n  -> record HBM bytes/launch for bench.py's roofline.traffic
if "--traffic-key" in sys.argv and "hbm_bytes_per_launch" in res:
    k = sys.argv[sys.argv.index("--traffic-key") + 1]
    root = Path(__file__).resolve().parent.parent
    dst = root / "profiles" / "pmc_traffic.json"
    db = json.loads(dst.read_text()) if dst.exists() else {}
    db[k] = {"bytes_per_launch": res["hbm_bytes_per_launch"], "source": str(d), "kernel_avg_ns": stats.get("avg_ns"),
             "fetch_size_kb": out.get("FETCH_SIZE"), "write_size_kb": out.get("WRITE_SIZE")}
    dst.write_text(json.dumps(db, indent=1) + "\n")
