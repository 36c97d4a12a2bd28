#!/bin/bash
# Lane-form occupancy: C3 with 1 WG/CU (128 KiB directories, prefetch) vs 2 WG/CU (<= 78 KiB).
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/sw5_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
run() {
    local name=$1; shift
    local envs=() args=()
    for a in "$@"; do if [[ $a == NFFACL_* ]]; then envs+=("$a"); else args+=("$a"); fi; done
    step "$name" env "${envs[@]}" timeout -k 10 300 $B "${args[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
step pytest bash -c "NFFACL_TUNE_DIR_KB=78 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'c3 or options or ragged' > $OUT/pytest.out 2>&1"
run c3_kb128 --config c3
run c3_kb78 NFFACL_TUNE_DIR_KB=78 --config c3
run c3_kb64 NFFACL_TUNE_DIR_KB=64 --config c3
run c3_kb40 NFFACL_TUNE_DIR_KB=40 --config c3
