#!/bin/bash
# SQ counter passes (instructions, waits, activity) of bench.py's C5 (or CFG)
# classify kernel under each NFFACL_TUNE_* variant, with summaries.
# usage: gpu_pmc_ab.sh TAG "NAME:VAR=VAL,VAR=VAL" ...   (CFG=c3 for another config)
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$1"; shift; mkdir -p "$OUT"
CFG=${CFG:-c5}
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-host --no-shapes --extra none --steps 10 --warmup 2 --config $CFG"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  for kv in ${envs//,/ }; do export "$kv"; done
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS \
      SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d "$OUT/${name}_sq" -o run --output-format csv -- $B > "$OUT/${name}_sq.out" 2>&1 \
      || { echo "sq $name failed"; tail -5 "$OUT/${name}_sq.out"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT \
      SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/${name}_sq2" -o run --output-format csv -- $B > "$OUT/${name}_sq2.out" 2>&1 \
      || { echo "sq2 $name failed"; tail -5 "$OUT/${name}_sq2.out"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum \
      -d "$OUT/${name}_tcc" -o run --output-format csv -- $B > "$OUT/${name}_tcc.out" 2>&1 \
      || { echo "tcc $name failed"; tail -5 "$OUT/${name}_tcc.out"; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/${name}_trace" -o run --output-format csv -- $B \
      > "$OUT/${name}_trace.out" 2>&1 || { echo "trace $name failed"; exit 1; }
  for kv in ${envs//,/ }; do unset "${kv%%=*}"; done
  python3 - "$OUT" "$name" <<'PY'
import collections, csv, json, sys
from pathlib import Path
out, name = Path(sys.argv[1]), sys.argv[2]
agg = collections.defaultdict(list)
for sub in ("sq", "sq2", "tcc"):
    for f in (out / f"{name}_{sub}").rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "k_indexed" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
w = m["SQ_WAVES"]; wc = m["SQ_WAVE_CYCLES"]
res = {"variant": name, "per_wave": {k: round(m[k] / w) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD")},
       "of_wave_cycles": {k: round(m[k] / wc, 3) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS")},
       "lds_bank_conflict": m.get("SQ_LDS_BANK_CONFLICT"), "grbm_gui_active": m.get("GRBM_GUI_ACTIVE"), "wave_cycles_per_wave": round(wc / w),
       "tcp_tcc_read_req": m.get("TCP_TCC_READ_REQ_sum"),
       "l2_hit": round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3) if m.get("TCC_HIT_sum") else None,
       "ta_busy_per_cu_cycle": round(m["TA_TA_BUSY_sum"] / 256 / (m["GRBM_GUI_ACTIVE"] / 8), 3) if m.get("TA_TA_BUSY_sum") else None}
for f in (out / f"{name}_trace").rglob("*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if "k_indexed" in r["Name"]:
            res["kernel_avg_ms"] = round(float(r["AverageNs"]) / 1e6, 4)
print(json.dumps(res))
json.dump(res, open(out / f"{name}_summary.json", "w"))
PY
done
