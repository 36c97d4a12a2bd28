#!/bin/bash
# Round 4: C5 / C3 with more workgroups than CUs (NFFACL_TUNE_PER_CU 2 / 4:
# later-starting workgroups then take a smaller share), alone.  usage: gpu_r4cc.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for c in c5 c3; do
  timeout -k 10 600 python tools/ab_env.py $c 4 base=NFFACL_AB:0 pc2=NFFACL_TUNE_PER_CU:2 pc4=NFFACL_TUNE_PER_CU:4 \
      > "$OUT/ab_${c}_per_cu.json" 2> "$OUT/ab_$c.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],{k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_${c}_per_cu.json"
done
