#!/bin/bash
# Burst / scalar call shapes (bench.py call_shapes, C2 rules) per environment
# variant, alternating, REPS times.  usage: gpu_burst_ab.sh TAG REPS SHAPES NAME=VAR:VAL[,VAR:VAL] ...
# SHAPES: NFFACL_BENCH_SHAPES, e.g. "burst:16:32:1.5,burst:32:32:1.5"
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$1"; REPS=$2; SH=$3; shift 3; mkdir -p "$OUT"; cd "$R"
for rep in $(seq $REPS); do for spec in "$@"; do
  name=${spec%%=*}; kv=${spec#*=}; envs=()
  IFS=, read -ra pairs <<< "$kv"
  for p in "${pairs[@]}"; do [ -n "$p" ] && envs+=("${p%%:*}=${p#*:}"); done
  env "${envs[@]}" NFFACL_BENCH_SHAPES="$SH" timeout -k 10 300 python bench.py --config c2 --extra none --no-host \
      --steps 5 --warmup 2 > "$OUT/${name}_$rep.json" 2> "$OUT/${name}_$rep.err" || { echo "$name failed"; tail -5 "$OUT/${name}_$rep.err"; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().splitlines()[-1])
cs=d.get('call_shapes',{}).get('c2',d.get('call_shapes',{}))
print(sys.argv[2], {k:(v.get('mpps'),v.get('lat_us_p50'),v.get('wrong')) for k,v in cs.items() if isinstance(v,dict)})" "$OUT/${name}_$rep.json" "$name $rep"
done; done
