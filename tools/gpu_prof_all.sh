#!/bin/bash
# Profiles of every config: tools/gpu_prof.sh (kernel trace + HBM / SQ / TCC / TA
# counter passes) for C5, C3 and C2, then their summaries.  usage: gpu_prof_all.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; cd "$R"
for c in c5 c3 c2; do
  bash tools/gpu_prof.sh "${T}_$c" --config $c || { echo "prof $c failed"; exit 1; }
  python3 tools/pmc_summary.py "gpurun_out/prof_${T}_$c" k_indexed > "gpurun_out/prof_${T}_$c/pmc_summary.json" || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d.get('trace'), d.get('hbm_bytes_per_launch'), d.get('per_wave'), d.get('l2_hit_rate'))" "gpurun_out/prof_${T}_$c/pmc_summary.json"
done
