#!/bin/bash
# Scalar-call path on the GPU: its tests, the thread sweep of
# tools/service_bench (built beforehand on the CPU: T threads x one-packet
# L3ACLPort calls through the C++ mirror's flow::ACLSplitter, every answer
# checked against the oracle), then the batcher / mirror / parity suites.
# usage: gpu_service.sh TAG [CFG]
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/service_$1"; CFG=${2:-c2}; mkdir -p "$OUT"; cd "$R"
PT="python -u -m pytest -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_service.py tests/test_reload.py > "$OUT/pytest1.out" 2>&1
rc=$?; echo "pytest1 exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
python tools/service_bench.py "$OUT/in" "$CFG" || exit 1
for t in 1 4 16 32 64; do
  timeout -k 10 60 ./tools/service_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" "$OUT/in/expect.bin" $t 3 >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err"
  rc=$?; echo "bench $t exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
done
rm -rf "$OUT/in"
timeout -k 10 900 $PT tests/test_batcher.py tests/test_cpp_mirror.py tests/test_gpu_parity.py > "$OUT/pytest2.out" 2>&1
rc=$?; echo "pytest2 exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
