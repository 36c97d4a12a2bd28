#!/bin/bash
# HYBRID kernel variants: parity, then C5/C3 benches.  usage: gpu_flat.sh TAG
#   flat rounds R in {2,4} x directory budgets; per-lane walk U in {1,2} with LDS directories
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/flat_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
step pytest bash -c "timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'budgets or full_size_c5 or c3 or c5' > $OUT/pytest.out 2>&1"
for cfg in c5 c3; do
  for r in 2 4; do
    for kb in ${KBS:-512 1024 2048}; do
      step "flat_${cfg}_r${r}_$kb" bash -c "NFFACL_TUNE_FLAT=1 NFFACL_TUNE_ROUNDS=$r NFFACL_TUNE_DIR_KB=$kb timeout -k 10 300 $B --config $cfg --algo hybrid > $OUT/flat_${cfg}_r${r}_$kb.json 2> $OUT/flat_${cfg}_r${r}_$kb.err"
    done
  done
  for u in 1 2; do
    for kb in 64 128; do
      step "lane_${cfg}_u${u}_$kb" bash -c "NFFACL_TUNE_UNROLL=$u NFFACL_TUNE_DIR_KB=$kb timeout -k 10 300 $B --config $cfg --algo hybrid > $OUT/lane_${cfg}_u${u}_$kb.json 2> $OUT/lane_${cfg}_u${u}_$kb.err"
    done
  done
done
