#!/bin/bash
# Closing record on the committed tree: full GPU parity suite, smoke(), then the
# C1 and L2 bench lines at default flags.  usage: gpu_final3.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/final3_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest bash -c "timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.out 2>&1"
step smoke bash -c "timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $OUT/smoke.out 2>&1"
for cfg in c1 l2; do
  step "bench_$cfg" bash -c "timeout -k 10 600 python bench.py --config $cfg --cpu-seconds 10 > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err"
done
