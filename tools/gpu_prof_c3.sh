#!/bin/bash
# C3 profile: counter list, standard trace + PMC passes (gpu_prof.sh), then a
# texture-unit pass.  usage: gpu_prof_c3.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out/prof_${TAG}_c3"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > "$R/gpurun_out/prof_${TAG}_c3/counters_list.txt" 2>&1 || true
bash "$R/tools/gpu_prof.sh" "${TAG}_c3" --config c3 || exit $?
