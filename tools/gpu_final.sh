#!/bin/bash
# Round record on one GPU: the whole -m gpu suite, smoke(), bench.py as the
# driver runs it and at its defaults, and the scalar-call sweep at default
# settings.  usage: gpu_final.sh TAG
R="$GRAFT_REPO_ROOT"; TAG=$1; cd "$R"; OUT="$R/gpurun_out/final_$TAG"; mkdir -p "$OUT"
step() {  # name, timeout, command...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name exit $rc" >> "$OUT/steps.log"
    return $rc
}
step pytest_gpu 900 python -u -m pytest -m gpu -v --timeout 150 --timeout-method thread -p no:cacheprovider tests || exit 1
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step bench_driver_cmd 600 python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
step bench_default 600 python bench.py || exit 1
python tools/service_bench.py "$OUT/in" c2 || exit 1
# callers pinned to the GPU's NUMA node (the recommended deployment), then not pinned
for t in 1 4 16 32 64; do
  step svc_$t 60 env NFFACL_BENCH_PIN=1 ./tools/service_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" "$OUT/in/expect.bin" $t 3 || exit 1
  cat "$OUT/svc_$t.out" >> "$OUT/service_sweep.jsonl"
done
for t in 1 16 32; do
  step svc_u$t 60 ./tools/service_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" "$OUT/in/expect.bin" $t 3 || exit 1
  cat "$OUT/svc_u$t.out" >> "$OUT/service_sweep_unpinned.jsonl"
done
rm -rf "$OUT/in"
