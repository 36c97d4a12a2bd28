#!/bin/bash
# Round 4: burst consumer — idle waves napping between bell reads
# (NFFACL_TUNE_SVC_IDLE_NAPS 0 / 5 / 20) at 1 / 16 / 32 clones.  usage: gpu_r4o.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_service_burst.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
for nap in 0 5 20; do
  NFFACL_TUNE_SVC_IDLE_NAPS=$nap NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5,burst:32:32:1.5" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/shapes_nap$nap.json" 2> "$OUT/shapes_nap$nap.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('nap$nap',{k:(v['mpps'],v['lat_us_p50'],v['lat_us_p99'],v['consumer_poll_us'],v['consumer_group_us'],v['wrong']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/shapes_nap$nap.json"
done
