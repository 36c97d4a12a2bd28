#!/bin/bash
# Time one variant of tools/ab_env.py against several builds of libnffacl
# (separate processes, alternating).  usage: exp_libs.sh TAG REPS "CFG..." LIB...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/exp_$1"; REPS=$2; CFGS=$3; shift 3; mkdir -p "$OUT"; cd "$R"
for c in $CFGS; do for rep in $(seq $REPS); do for lib in "$@"; do
  NFFACL_LIB=$R/$lib timeout -k 10 300 python tools/ab_env.py $c 3 v=NFFACL_TUNE_FLAT:2 > "$OUT/${c}_$(basename $lib .so)_$rep.json" 2>/dev/null || exit 1
done; done; done
