#!/bin/bash
# Two-level directories: parity, then C3 lane-form budgets.  usage: gpu_sweep4.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/sw4_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host"
run() {  # name, env assignments..., then bench args
    local name=$1; shift
    local envs=() args=()
    for a in "$@"; do if [[ $a == NFFACL_* ]]; then envs+=("$a"); else args+=("$a"); fi; done
    step "$name" env "${envs[@]}" timeout -k 10 300 $B "${args[@]}" > "$OUT/$name.json" 2> "$OUT/$name.err"
}
step pytest bash -c "timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'hybrid or budgets or c3 or c5 or kats or options' > $OUT/pytest.out 2>&1"
run c3_kb128 --config c3
run c3_kb80 NFFACL_TUNE_DIR_KB=78 --config c3
run c3_kb64 NFFACL_TUNE_DIR_KB=64 --config c3
run c3_u32 NFFACL_TUNE_DIR16=0 --config c3
run c3_kb128_u2 NFFACL_TUNE_UNROLL=2 --config c3
