#!/bin/bash
# HYBRID flat-LDS form: parity, then in-process A/B of the table forms on C5 and C3.
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out/flatlds_$1"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest bash -c "timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'hybrid or c5 or c3 or frames' > $OUT/pytest.out 2>&1"
step ab_c5 bash -c "timeout -k 10 400 python tools/ab_env.py c5 5 flat_global=NFFACL_TUNE_FLAT:1 flat_lds=NFFACL_TUNE_FLAT:2 > $OUT/ab_c5.json 2> $OUT/ab_c5.err"
step ab_c3 bash -c "timeout -k 10 400 python tools/ab_env.py c3 5 lane=NFFACL_TUNE_FLAT:0 flat_lds=NFFACL_TUNE_FLAT:2 > $OUT/ab_c3.json 2> $OUT/ab_c3.err"
