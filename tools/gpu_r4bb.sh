#!/bin/bash
# Round 4: C2 / C5 batch kernel time alone, with a scalar and a burst
# service kept hot by caller threads, and after.
# usage: gpu_r4bb.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python tools/svc_overlap.py 4 > "$OUT/svc_overlap.json" 2> "$OUT/svc_overlap.err" || { tail -5 "$OUT/svc_overlap.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:d[k] for k in ('alone_ms','armed_ms','after_ms','slowdown_armed','calls_during')})" "$OUT/svc_overlap.json"
