#!/bin/bash
# Round record on one GPU: the whole -m gpu suite, smoke(), bench.py as the
# driver runs it and at its defaults (C2 + C3/C5 configs, host-inclusive,
# call shapes at C2/C3/C5).  Profiles: tools/gpu_prof.sh.  usage: gpu_final.sh TAG
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
