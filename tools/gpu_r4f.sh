#!/bin/bash
# Round 4: full GPU suite with the fine-slot / directory-density defaults, and
# env A/B of those defaults against the previous ones on C5 and C3.
# usage: gpu_r4f.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
for c in c5 c3; do
  timeout -k 10 600 python tools/ab_env.py $c 4 new=NFFACL_AB:0 old=NFFACL_TUNE_FINE_A:0,NFFACL_TUNE_DIR_PER_RULE:4 \
      dir4=NFFACL_TUNE_DIR_PER_RULE:4 nofine=NFFACL_TUNE_FINE_A:0 d8=NFFACL_TUNE_DIR_PER_RULE:8 \
      > "$OUT/ab_$c.json" 2> "$OUT/ab_$c.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], {k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_$c.json"
done
