#!/bin/bash
# Directory-budget / form sweep for C3 and C5 (HYBRID).  usage: gpu_sweep3.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/sw3_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
run() {  # name, env assignments..., then bench args
    local name=$1; shift
    local envs=() args=()
    for a in "$@"; do if [[ $a == NFFACL_* ]]; then envs+=("$a"); else args+=("$a"); fi; done
    step "$name" env "${envs[@]}" timeout -k 10 300 $B "${args[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run c3_kb48 NFFACL_TUNE_DIR_KB=48 --config c3
run c3_kb64 NFFACL_TUNE_DIR_KB=64 --config c3
run c3_kb96 NFFACL_TUNE_DIR_KB=96 --config c3
run c3_kb128 NFFACL_TUNE_DIR_KB=128 --config c3
run c5_lane NFFACL_TUNE_FLAT=0 --config c5
run c5_lane64 NFFACL_TUNE_FLAT=0 NFFACL_TUNE_DIR_KB=64 --config c5
run c5_kb512 NFFACL_TUNE_DIR_KB=512 NFFACL_TUNE_FLAT=1 --config c5
run c5_kb1024_r2 NFFACL_TUNE_DIR_KB=1024 NFFACL_TUNE_FLAT=1 NFFACL_TUNE_ROUNDS=2 --config c5
run c5_kb2048 NFFACL_TUNE_DIR_KB=2048 NFFACL_TUNE_FLAT=1 --config c5
