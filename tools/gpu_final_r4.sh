#!/bin/bash
# Round 4 final: the record (tools/gpu_final.sh) then the C5 profile again
# (the fine-grid default changed after prof_r4_c5).  usage: gpu_final_r4.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; cd "$R"
bash tools/gpu_final.sh "$T" || { cat "gpurun_out/final_$T/steps.log"; exit 1; }
cat "gpurun_out/final_$T/steps.log"
bash tools/gpu_prof.sh "${T}_c5" --config c5 || { echo "prof c5 failed"; exit 1; }
python3 tools/pmc_summary.py "gpurun_out/prof_${T}_c5" k_indexed > "gpurun_out/prof_${T}_c5/pmc_summary.json" || exit 1
