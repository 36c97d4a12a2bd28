#!/bin/bash
# parity of the stride-64 kernels under a forced load mode, then A/B.  usage: gpu_ab2.sh TAG MODE
TAG=$1; MODE=$2; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/ab2_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step parity bash -c "NFFACL_TUNE_COAL=$MODE timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_vlan.py -m gpu -q -x -p no:cacheprovider > $OUT/parity.out 2>&1"
step ab bash -c "timeout -k 10 600 python tools/ab.py c2 10 > $OUT/ab_c2.json 2> $OUT/ab_c2.err"
step ab1 bash -c "timeout -k 10 600 python tools/ab.py c2 10 > $OUT/ab_c2_b.json 2> $OUT/ab_c2_b.err"
