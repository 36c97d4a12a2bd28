#!/bin/bash
# flat-LDS tuning A/B: directory budget (compile) and workgroup shape (launch).
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out/flattune_$1"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
for cfg in c5 c3; do
  step "ab_$cfg" bash -c "timeout -k 10 500 python tools/ab_env.py $cfg 4 d128=NFFACL_TUNE_DIR_KB:128 d96=NFFACL_TUNE_DIR_KB:96 d64=NFFACL_TUNE_DIR_KB:64 d64_2x512=NFFACL_TUNE_DIR_KB:64,NFFACL_TUNE_BLOCK:512,NFFACL_TUNE_PER_CU:2 d48_3x256=NFFACL_TUNE_DIR_KB:48,NFFACL_TUNE_BLOCK:256,NFFACL_TUNE_PER_CU:3 > $OUT/ab_$cfg.json 2> $OUT/ab_$cfg.err"
done
