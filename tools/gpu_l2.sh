#!/bin/bash
# L2 parity + bench.  usage: gpu_l2.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out/l2_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest bash -c "timeout -k 10 900 python -m pytest tests/test_l2.py tests/test_gpu_parity.py -m gpu -q -x -p no:cacheprovider > $OUT/pytest.out 2>&1"
step bench bash -c "timeout -k 10 600 python bench.py --config l2 --steps 20 --cpu-seconds 3 > $OUT/bench_l2.json 2> $OUT/bench_l2.err"
