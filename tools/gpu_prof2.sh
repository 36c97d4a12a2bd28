#!/bin/bash
# Profile the hybrid variants of C5 (flat) and C3 (per-lane walk).  usage: gpu_prof2.sh TAG
R="$GRAFT_REPO_ROOT"; TAG=$1
export NFFACL_TUNE_DIR_KB=1024 NFFACL_TUNE_FLAT=1
bash "$R/tools/gpu_prof.sh" "${TAG}_c5flat" --config c5 --algo hybrid || exit $?
unset NFFACL_TUNE_FLAT
export NFFACL_TUNE_DIR_KB=128 NFFACL_TUNE_UNROLL=2
bash "$R/tools/gpu_prof.sh" "${TAG}_c3lane" --config c3 --algo hybrid || exit $?
