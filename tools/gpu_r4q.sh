#!/bin/bash
# Round 4: burst call shapes with the mailboxes on the device's NUMA node
# (default) or under the caller's default policy (NFFACL_TUNE_SVC_NODE=0).
# usage: gpu_r4q.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for nd in 1 0; do
  NFFACL_TUNE_SVC_NODE=$nd NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5,scalar:1:0:1.0,scalar:32:0:1.0" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/shapes_node$nd.json" 2> "$OUT/shapes_node$nd.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('node$nd',{k:(v['mpps'],v['lat_us_p50'],v['lat_us_p99'],v['consumer_poll_us'],v['consumer_group_us'],v['wrong']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/shapes_node$nd.json"
done
