#!/bin/bash
# Parity of the HYBRID path, then C3/C5 benches (auto = hybrid vs indexed)
# [+ directory-budget sweep if SWEEP=1].  usage: gpu_hyb.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/hyb_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
step pytest bash -c "timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'hybrid or HYBRID or c3 or c5 or kats or ragged or options' > $OUT/pytest.out 2>&1"
for cfg in c5 c3; do
  for algo in auto indexed; do
    step "bench_${cfg}_$algo" bash -c "timeout -k 10 300 $B --config $cfg --algo $algo > $OUT/bench_${cfg}_$algo.json 2> $OUT/bench_${cfg}_$algo.err"
  done
done
if [ "${SWEEP:-0}" = 1 ]; then
  for kb in 32 96 128; do
    for cfg in c5 c3; do
      step "sweep_${cfg}_$kb" bash -c "NFFACL_TUNE_DIR_KB=$kb timeout -k 10 300 $B --config $cfg > $OUT/sweep_${cfg}_$kb.json 2> $OUT/sweep_${cfg}_$kb.err"
    done
  done
fi
