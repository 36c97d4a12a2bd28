#!/bin/bash
# Full GPU parity suite, then default benches (C2, C3, C5) and per-lane walk variants for C3.
# usage: gpu_round2.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/r2_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
step pytest bash -c "timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.out 2>&1"
for cfg in c2 c3 c5; do
  step "bench_$cfg" bash -c "timeout -k 10 300 $B --config $cfg > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err"
done
for u in 1; do
  step "c3_u$u" bash -c "NFFACL_TUNE_UNROLL=$u timeout -k 10 300 $B --config c3 > $OUT/c3_u$u.json 2> $OUT/c3_u$u.err"
done
