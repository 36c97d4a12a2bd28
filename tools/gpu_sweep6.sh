#!/bin/bash
# Flat form with split address slots: parity, then C5 over split widths / directory budgets.
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/sw6_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
run() {
    local name=$1; shift
    local envs=() args=()
    for a in "$@"; do if [[ $a == NFFACL_* ]]; then envs+=("$a"); else args+=("$a"); fi; done
    step "$name" env "${envs[@]}" timeout -k 10 300 $B "${args[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
step pytest bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'hybrid or budgets or c5 or c3 or kats' > $OUT/pytest.out 2>&1"
run c5_q4_1m --config c5
run c5_q0_1m NFFACL_TUNE_SPLIT=0 --config c5
run c5_q4_2m NFFACL_TUNE_DIR_KB=2048 NFFACL_TUNE_FLAT=1 --config c5
run c5_q4_4m NFFACL_TUNE_DIR_KB=4096 NFFACL_TUNE_FLAT=1 --config c5
run c5_q6_2m NFFACL_TUNE_SPLIT=6 NFFACL_TUNE_DIR_KB=2048 NFFACL_TUNE_FLAT=1 --config c5
run c5_q2_1m NFFACL_TUNE_SPLIT=2 --config c5
