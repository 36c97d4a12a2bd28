#!/bin/bash
# L2 parity, then in-process A/B of the header load (lane-contiguous vs row piece).
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out/l2coal_$1"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest bash -c "timeout -k 10 900 python -u -m pytest tests/test_l2.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'gpu_ or c2 or kats or ragged' > $OUT/pytest.out 2>&1"
step ab bash -c "timeout -k 10 300 python tools/ab_env.py l2 6 coal=NFFACL_TUNE_L2_COAL:1 row=NFFACL_TUNE_L2_COAL:0 > $OUT/ab_l2.json 2> $OUT/ab_l2.err"
