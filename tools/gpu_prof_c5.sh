#!/bin/bash
# C5 profile of the committed kernel (tools/gpu_prof.sh) and its summary.  usage: gpu_prof_c5.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; cd "$R"
bash tools/gpu_prof.sh "${T}_c5" --config c5 || { echo "prof c5 failed"; exit 1; }
python3 tools/pmc_summary.py "gpurun_out/prof_${T}_c5" k_indexed > "gpurun_out/prof_${T}_c5/pmc_summary.json" || exit 1
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['trace'], d.get('hbm_bytes_per_launch'), d.get('per_wave'), d.get('l2_hit_rate'))" "gpurun_out/prof_${T}_c5/pmc_summary.json"
