#!/usr/bin/env python3
"""Mean per-dispatch SQ counters of one kernel from a rocprofv3 --pmc run
directory (any layout: every *counter_collection.csv below it).
usage: pmc_sq.py DIR [kernel substring]"""
import collections
import csv
import json
import sys
from pathlib import Path

d = Path(sys.argv[1])
key = sys.argv[2] if len(sys.argv) > 2 else "k_indexed"
agg = collections.defaultdict(list)
for f in d.rglob("*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: sum(v) / len(v) for k, v in agg.items()}
w = out.get("SQ_WAVES")
res = {"dir": str(d), "kernel": key, "dispatches": max((len(v) for v in agg.values()), default=0), "mean": out}
if w:
    res["per_wave"] = {k: v / w for k, v in out.items() if k != "SQ_WAVES"}
print(json.dumps(res))
