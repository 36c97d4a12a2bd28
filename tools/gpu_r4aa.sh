#!/bin/bash
# Round 4: scalar consumer, the round-3 poll order (NFFACL_EXP_SVCSTAT=16
# build) against the current one, alternating.  usage: gpu_r4aa.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for rep in 1 2; do for lib in libnffacl build_exp/svc16; do
  n=$(basename $lib)_$rep
  NFFACL_LIB=$R/nff-go_amd/$lib.so NFFACL_BENCH_SHAPES="scalar:1:0:1.0,scalar:16:0:1.0,scalar:32:0:1.5" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/$n.json" 2> "$OUT/$n.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('$n',{k:(v['mpps'],v['lat_us_p50'],v['wrong']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/$n.json"
done; done
