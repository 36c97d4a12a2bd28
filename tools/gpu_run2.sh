#!/bin/bash
# GPU session 2: parity tests (linear + indexed), bench both algorithms,
# kernel-trace profile and HBM PMC passes of the headline bench.
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() {  # name, timeout, command...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.out" 2> "gpurun_out/$name.err"
    local rc=$?
    echo "$name exit $rc" >> gpurun_out/steps.log
    return $rc
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step bench_indexed 600 python bench.py --steps 20 --warmup 3 --algo indexed || exit $?
step bench_linear 600 python bench.py --steps 10 --warmup 2 --algo linear --no-cpu-baseline --no-host || exit $?
cd /tmp && export TMPDIR=/tmp
step prof_trace 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --algo indexed --no-cpu-baseline --no-host || exit $?
step prof_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/prof_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --algo indexed --no-cpu-baseline --no-host || exit $?
step prof_write 600 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/prof_write" -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --algo indexed --no-cpu-baseline --no-host || exit $?
