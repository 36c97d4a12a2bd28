#!/bin/bash
# Parity subset, then one-process interleaved A/B of NFFACL_TUNE_* variants.
# usage: gpu_ab.sh TAG "PYTEST -k EXPR" CFG "VARIANTS..." [CFG "VARIANTS..."]...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab_$1"; K="$2"; shift 2; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "$K" --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.out" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
while [ $# -ge 2 ]; do
  c=$1; v=$2; shift 2
  timeout -k 10 600 python tools/ab_env.py "$c" 6 $v > "$OUT/ab_$c.json" 2> "$OUT/ab_$c.err"
  rc=$?; echo "ab $c exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
done
