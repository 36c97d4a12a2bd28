#!/bin/bash
# Round 4: burst calls with the kernels reading the mailboxes through the
# hipHostGetDevicePointer alias (default) or the host pointer itself
# (NFFACL_TUNE_SVC_HOSTPTR=1), host-side phase trace on.  usage: gpu_r4t.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for hp in 0 1; do
  NFFACL_TUNE_SVC_HOSTPTR=$hp NFFACL_TUNE_SVC_TRACE=1 NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/hostptr$hp.json" 2> "$OUT/hostptr$hp.err" || exit 1
  grep "service trace" "$OUT/hostptr$hp.err"
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('hostptr$hp',{k:(v['mpps'],v['lat_us_p50'],v['consumer_group_us'],v['wrong']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/hostptr$hp.json"
done
