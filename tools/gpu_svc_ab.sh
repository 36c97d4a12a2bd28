#!/bin/bash
# Scalar-call sweep A/B: tools/service_bench0 (linked against a baseline
# libnffacl under build_prev/svc0) and tools/service_bench (the working
# library), alternating per thread count.  usage: gpu_svc_ab.sh TAG
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/svcab_$1"; mkdir -p "$OUT"; cd "$R"
python tools/service_bench.py "$OUT/in" c2 || exit 1
for rep in 1 2; do for t in 1 16 32; do for b in service_bench0 service_bench; do
  timeout -k 10 60 ./tools/$b "$OUT/in/rules.conf" "$OUT/in/slots.bin" "$OUT/in/expect.bin" $t 3 > "$OUT/r.json" 2>> "$OUT/err.log" || exit 1
  echo "{\"bin\": \"$b\", \"r\": $(cat $OUT/r.json)}" >> "$OUT/sweep.jsonl"
done; done; done
rm -rf "$OUT/in"
