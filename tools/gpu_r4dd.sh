#!/bin/bash
# Round 4: batch kernels beside busy consumers with the default grid and with
# 4 workgroups per CU (NFFACL_TUNE_PER_CU=4).  usage: gpu_r4dd.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for pc in 0 4; do
  if [ $pc = 0 ]; then unset NFFACL_TUNE_PER_CU; else export NFFACL_TUNE_PER_CU=$pc; fi
  timeout -k 10 300 python tools/svc_overlap.py 4 > "$OUT/svc_overlap_pc$pc.json" 2> "$OUT/svc_overlap_pc$pc.err" || { tail -5 "$OUT/svc_overlap_pc$pc.err"; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print('pc$pc',{k:d[k] for k in ('alone_ms','armed_ms','after_ms','slowdown_armed')})" "$OUT/svc_overlap_pc$pc.json"
done
