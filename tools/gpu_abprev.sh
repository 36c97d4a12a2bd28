#!/bin/bash
# Current library vs nff-go_amd/libnffacl_prev.so (a build of the previous
# variant), alternating processes on one box, after a parity subset.
# usage: gpu_abprev.sh TAG "pytest -k expr" CONFIG [CONFIG...]
TAG=$1; K=$2; shift 2; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/abprev_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k '$K' > $OUT/pytest.out 2>&1"
for cfg in "$@"; do
  for i in 1 2; do
    step "${cfg}_prev$i" bash -c "NFFACL_LIB=$R/nff-go_amd/libnffacl_prev.so timeout -k 10 300 python tools/ab_env.py $cfg 4 x= > $OUT/${cfg}_prev$i.json 2> $OUT/${cfg}_prev$i.err"
    step "${cfg}_new$i" bash -c "timeout -k 10 300 python tools/ab_env.py $cfg 4 x= > $OUT/${cfg}_new$i.json 2> $OUT/${cfg}_new$i.err"
  done
done
