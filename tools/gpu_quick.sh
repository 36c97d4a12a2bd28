#!/bin/bash
# Parity subset + default benches.  usage: gpu_quick.sh TAG [pytest -k expr]
TAG=$1; K=${2:-"kats or options or c3 or c5 or c2 or ragged or header"}; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/q_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
step pytest bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k '$K' > $OUT/pytest.out 2>&1"
for cfg in ${CFGS:-c2 c3 c5}; do
  step "bench_$cfg" bash -c "timeout -k 10 300 $B --config $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err"
done
