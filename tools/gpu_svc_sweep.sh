#!/bin/bash
# Scalar-call tests, then tools/service_bench thread sweeps per variant
# (NFFACL_TUNE_SVC_* settings).  usage: gpu_svc_sweep.sh TAG CFG "VAR=VAL ..." ["VAR=VAL ..."]...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/svcsweep_$1"; CFG=$2; shift 2; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
    tests/test_service.py tests/test_reload.py > "$OUT/pytest.out" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
python tools/service_bench.py "$OUT/in" "$CFG" || exit 1
for v in "$@"; do for t in 1 4 16 32 64; do
  env $v timeout -k 10 60 ./tools/service_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" "$OUT/in/expect.bin" $t 3 > "$OUT/r.json" 2>> "$OUT/sweep.err"
  rc=$?; echo "bench [$v] $t exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
  echo "{\"variant\": \"$v\", \"r\": $(cat $OUT/r.json)}" >> "$OUT/sweep.jsonl"
done; done
rm -rf "$OUT/in"
