#!/bin/bash
# Measure every BASELINE config on one GPU, then rehearse the N=2 bench path
# (2 ranks on this one GPU over gloo, incl. the scatter-inclusive curve).
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/configs_$1"; mkdir -p "$OUT"; cd "$R"
run() { local name=$1; shift; timeout -k 10 600 python bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; return $rc; }
run c1 --config c1 --no-host --cpu-seconds 5 || exit $?
run c1_indexed --config c1 --algo indexed --no-host --no-cpu-baseline || exit $?
run c5_indexed --config c5 --no-host --cpu-seconds 10 || exit $?
run c3_indexed --config c3 --packets 4194304 --cpu-seconds 5 || exit $?
run c2_linear --algo linear --no-host --no-cpu-baseline --steps 5 || exit $?
NFFACL_BENCH_ONE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 \
  --packets 1048576 --no-host > "$OUT/n2_gloo.json" 2> "$OUT/n2_gloo.err"
rc=$?; echo "n2_gloo exit $rc" >> "$OUT/steps.log"; exit $rc
