#!/bin/bash
# Default bench (region timing, K=100, CPU baseline) for C2/C3/C5, then the N=2
# bench path rehearsed on this one GPU (2 ranks over gloo).  usage: gpu_final2.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/final2_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step bench_default bash -c "timeout -k 10 600 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err"
for cfg in c3 c5; do
  step "bench_$cfg" bash -c "timeout -k 10 600 python bench.py --config $cfg --cpu-seconds 10 > $OUT/bench_$cfg.json 2> $OUT/bench_$cfg.err"
done
step n2_gloo bash -c "NFFACL_BENCH_ONE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --packets 1048576 --no-host \
  > $OUT/n2_gloo.json 2> $OUT/n2_gloo.err"
