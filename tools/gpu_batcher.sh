#!/bin/bash
# Host-ingest sweep of nffacl_batcher (tools/batcher_bench.cpp).  usage: gpu_batcher.sh TAG
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/batcher_$1"; mkdir -p "$OUT"; cd "$R"
python tools/batcher_bench.py /tmp/bb || exit 1
g++ -O2 -std=c++17 -pthread -Iinclude tools/batcher_bench.cpp -Lnff-go_amd -lnffacl -Wl,-rpath,"$R/nff-go_amd" -o /tmp/bb/batcher_bench || exit 1
for cfg in "1 32 4096 50" "4 32 4096 50" "8 32 8192 100" "16 32 16384 100" "16 32 65536 200" "32 32 65536 200" "16 8 16384 100" "8 32 1024 20"; do
  set -- $cfg
  timeout -k 10 60 /tmp/bb/batcher_bench /tmp/bb/rules.conf /tmp/bb/slots.bin 80 $1 $2 $3 $4 3 >> "$OUT/results.jsonl" 2>> "$OUT/err.log"
  rc=$?; echo "cfg $cfg exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc
done
