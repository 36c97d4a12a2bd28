#!/bin/bash
# Batcher tests, then the host-ingest sweep (tools/batcher_bench.cpp, built
# beforehand on the CPU): T threads x bursts of B packets, synchronous
# submit + wait per burst (B = 1: SetSeparator's per-packet call shape).
# usage: gpu_batcher.sh TAG
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/batcher_$1"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "batcher or cpp_mirror or swap" --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.out" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
python tools/batcher_bench.py "$OUT/in" || exit 1
for tb in 1:1 8:1 32:1 64:1 1:32 4:32 16:32 32:32 64:32; do
  t=${tb%:*}; b=${tb#*:}
  timeout -k 10 60 ./tools/batcher_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" 80 $t $b 8192 100 2 >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err"
  rc=$?; echo "bench $tb exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
done
rm -rf "$OUT/in"
