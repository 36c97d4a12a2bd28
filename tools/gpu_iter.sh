#!/bin/bash
# One GPU iteration: parity tests, the headline bench, then a profile.
# usage: bash tools/gpu_iter.sh <tag> [pytest -k expr]
R="$GRAFT_REPO_ROOT"
TAG=$1; K=${2:-}
OUT="$R/gpurun_out/iter_$TAG"
mkdir -p "$OUT"
cd "$R"
if [ -n "$K" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider -k "$K" > "$OUT/pytest.out" 2>&1
else
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest.out" 2>&1
fi
rc=$?; echo "pytest exit $rc" >> "$OUT/steps.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc" >> "$OUT/steps.log"
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_prof.sh "$TAG" --algo indexed
