#!/bin/bash
# Round 4: whole GPU suite after the one-round-trip polls, then the call-shape
# sweep (bursts 1 / 16 / 24 / 32 clones, scalar 1 / 16 / 32 threads).  usage: gpu_r4z.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5,burst:24:32:1.5,burst:32:32:1.5,scalar:1:0:1.0,scalar:16:0:1.0,scalar:32:0:1.5" \
  timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
    > "$OUT/shapes.json" 2> "$OUT/shapes.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print({k:(v['mpps'],v['lat_us_p50'],v['lat_us_p99'],v['wrong']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/shapes.json"
