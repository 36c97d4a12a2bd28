#!/bin/bash
# Round 4: burst consumer answer -> next-request gap (NFFACL_EXP_SVCSTAT build:
# consumer_poll_us = that gap, hot waves only), then the round's kernel
# profiles (tools/gpu_prof_r4.sh).  usage: gpu_r4r.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
NFFACL_LIB=$R/nff-go_amd/build_exp/svcstat.so NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5" \
  timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
    > "$OUT/shapes_svcstat.json" 2> "$OUT/shapes_svcstat.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print({k:(v['mpps'],v['lat_us_p50'],v['consumer_poll_us'],v['consumer_group_us'],v['polls_per_call']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/shapes_svcstat.json"
bash tools/gpu_prof_r4.sh r4 || exit 1
