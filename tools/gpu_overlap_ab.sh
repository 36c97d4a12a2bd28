#!/bin/bash
# tools/svc_overlap.py (batch kernels alone / beside busy resident consumers)
# once per environment variant.  usage: gpu_overlap_ab.sh TAG NAME=VAR:VAL[,VAR:VAL] ...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$1"; shift; mkdir -p "$OUT"; cd "$R"
for spec in "$@"; do
  name=${spec%%=*}; kv=${spec#*=}
  envs=()
  IFS=, read -ra pairs <<< "$kv"
  for p in "${pairs[@]}"; do [ -n "$p" ] && envs+=("${p%%:*}=${p#*:}"); done
  env "${envs[@]}" timeout -k 10 240 python tools/svc_overlap.py > "$OUT/overlap_$name.json" 2> "$OUT/overlap_$name.err" \
      || { echo "overlap $name failed"; tail -20 "$OUT/overlap_$name.err"; exit 1; }
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[2], 'alone', {k: round(v, 4) for k, v in d['alone_ms'].items()}, 'armed', {k: round(v, 4) for k, v in d['armed_ms'].items()}, d['slowdown_armed'])" "$OUT/overlap_$name.json" "$name"
done
