#!/bin/bash
# A/B of bench.py's timing modes (per-launch event pairs vs one region pair) on C2 and C5.
# usage: gpu_timing.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/timing_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
B="python bench.py --warmup 3 --no-cpu-baseline --no-host"
for rep in 1 2; do
  for mode in launch region; do
    for st in 20 100; do
      step "c2_${mode}_${st}_$rep" bash -c "timeout -k 10 300 $B --steps $st --timing $mode > $OUT/c2_${mode}_${st}_$rep.json 2> $OUT/c2_${mode}_${st}_$rep.err"
    done
  done
done
for mode in launch region; do
  step "c5_$mode" bash -c "timeout -k 10 300 $B --config c5 --timing $mode > $OUT/c5_$mode.json 2> $OUT/c5_$mode.err"
done
