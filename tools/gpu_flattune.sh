#!/bin/bash
# flat-LDS tuning A/B: rounds in flight x directory budget (compile + launch knobs).
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out/flattune_$1"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
for cfg in c5 c3; do
  step "ab_$cfg" bash -c "timeout -k 10 500 python tools/ab_env.py $cfg 4 r2_d128=NFFACL_TUNE_ROUNDS:2 r4_d120=NFFACL_TUNE_ROUNDS:4,NFFACL_TUNE_DIR_KB:120 r2_d120=NFFACL_TUNE_ROUNDS:2,NFFACL_TUNE_DIR_KB:120 r4_d104=NFFACL_TUNE_ROUNDS:4,NFFACL_TUNE_DIR_KB:104 > $OUT/ab_$cfg.json 2> $OUT/ab_$cfg.err"
done
