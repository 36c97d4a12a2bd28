#!/bin/bash
# Round 4: burst callers spinning on all 32 response words (default) or on
# the last one first (NFFACL_TUNE_SVC_SPIN1=1).  usage: gpu_r4x.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for sp in 0 1; do
  NFFACL_TUNE_SVC_SPIN1=$sp NFFACL_TUNE_SVC_TRACE=1 NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5,burst:32:32:1.5" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/spin1_$sp.json" 2> "$OUT/spin1_$sp.err" || exit 1
  grep "service trace" "$OUT/spin1_$sp.err"
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('spin1_$sp',{k:(v['mpps'],v['lat_us_p50'],v['wrong']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/spin1_$sp.json"
done
