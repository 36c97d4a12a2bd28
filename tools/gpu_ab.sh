#!/bin/bash
# GPU suite, then interleaved A/B of launch variants.  usage: gpu_ab.sh TAG CFG...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab_$1"; shift; mkdir -p "$OUT"; cd "$R"
make -s -C tests/cpp > "$OUT/make.out" 2>&1 || exit 1
timeout -k 10 1200 python -m pytest tests -m gpu -q -x -p no:cacheprovider > "$OUT/pytest.out" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
for c in "$@"; do
  timeout -k 10 600 python tools/ab.py "$c" 10 > "$OUT/ab_$c.json" 2> "$OUT/ab_$c.err"
  rc=$?; echo "ab $c exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --config l2 --steps 20 --cpu-seconds 5 > "$OUT/bench_l2.json" 2> "$OUT/bench_l2.err"
rc=$?; echo "bench l2 exit $rc" >> "$OUT/steps.log"; exit $rc
