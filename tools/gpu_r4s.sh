#!/bin/bash
# Round 4: host-side phase times of burst calls (NFFACL_TUNE_SVC_TRACE=1:
# post / wait per call, printed when the service is destroyed) at 1 and 16
# clones, C2 rules.  usage: gpu_r4s.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for sh in "burst:1:32:1.5" "burst:16:32:1.5"; do
  n=${sh//:/_}
  NFFACL_TUNE_SVC_TRACE=1 NFFACL_BENCH_SHAPES="$sh" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/trace_$n.json" 2> "$OUT/trace_$n.err" || exit 1
  grep "service trace" "$OUT/trace_$n.err"
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print({k:(v['mpps'],v['lat_us_p50'],v['consumer_group_us']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/trace_$n.json"
done
