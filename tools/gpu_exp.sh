#!/bin/bash
# One GPU call, two experiments: the kernel-library A/B of tools/exp_libs.sh
# (CFGS, libs) and a tools/service_bench thread sweep per NFFACL_TUNE_SVC_*
# variant (no test pass first).  usage: gpu_exp.sh TAG "CFGS" "LIB..." "VAR=VAL"...
R="$GRAFT_REPO_ROOT"; TAG=$1; CFGS=$2; LIBS=$3; shift 3; cd "$R"
OUT="$R/gpurun_out/svcsweep_$TAG"; mkdir -p "$OUT"
python tools/service_bench.py "$OUT/in" c2 || exit 1
for v in "$@"; do for t in 1 4 16 32 64; do
  env $v timeout -k 10 60 ./tools/service_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" "$OUT/in/expect.bin" $t 3 > "$OUT/r.json" 2>> "$OUT/sweep.err"
  rc=$?; echo "bench [$v] $t exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
  echo "{\"variant\": \"$v\", \"r\": $(cat $OUT/r.json)}" >> "$OUT/sweep.jsonl"
done; done
rm -rf "$OUT/in"
[ -n "$CFGS" ] && bash tools/exp_libs.sh "$TAG" 3 "$CFGS" $LIBS
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline > "$R/gpurun_out/svcsweep_$TAG/bench.json" 2> "$R/gpurun_out/svcsweep_$TAG/bench.err" || exit 1
fi
