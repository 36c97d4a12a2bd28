#!/bin/bash
# Measure every BASELINE config on one GPU (C1, C2 linear+indexed, C3 frames, C5).
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/configs_$1"; mkdir -p "$OUT"; cd "$R"
run() { local name=$1; shift; timeout -k 10 600 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; return $rc; }
run c1_indexed --config c1 --no-host --cpu-seconds 5 || exit $?
run c1_linear --config c1 --algo linear --no-host --no-cpu-baseline || exit $?
run c5_indexed --config c5 --no-host --cpu-seconds 10 || exit $?
run c3_indexed --config c3 --packets 4194304 || exit $?
run c2_linear --algo linear --no-host --no-cpu-baseline --steps 5 || exit $?
