#!/bin/bash
# Whole -m gpu suite and smoke() on the tree as committed.  usage: gpu_verify.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.out" 2>&1 || { tail -20 "$OUT/smoke.out"; exit 1; }
tail -1 "$OUT/smoke.out"
# optional: BENCH=1 also runs bench.py as the driver does (K = 20, W = 5)
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.out" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().splitlines()[-1]);print(json.dumps(d['summary']))" "$OUT/bench.out"
fi
