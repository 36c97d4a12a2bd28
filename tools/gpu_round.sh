#!/bin/bash
# tests -> bench c2 / l2 -> batcher sweep [-> A/B c2 if AB=1].  usage: gpu_round.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/round_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step make make -s -C tests/cpp
step pytest bash -c "timeout -k 10 1200 python -m pytest tests -m gpu -q -x -p no:cacheprovider > $OUT/pytest.out 2>&1"
step bench_c2 bash -c "timeout -k 10 600 python bench.py --steps 20 > $OUT/bench_c2.json 2> $OUT/bench_c2.err"
step bench_l2 bash -c "timeout -k 10 600 python bench.py --config l2 --steps 20 --cpu-seconds 5 > $OUT/bench_l2.json 2> $OUT/bench_l2.err"
step batcher bash tools/gpu_batcher.sh "$TAG"
if [ "${AB:-0}" = 1 ]; then step ab bash -c "timeout -k 10 600 python tools/ab.py c2 8 > $OUT/ab_c2.json 2> $OUT/ab_c2.err"; fi
