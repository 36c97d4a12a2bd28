#!/bin/bash
# Profile the headline bench: kernel trace + stats, HBM PMC passes (FETCH_SIZE,
# WRITE_SIZE in separate passes), SQ instruction/stall counters.
# usage: bash tools/gpu_prof.sh <tag> [bench args...]
R="$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
step() {  # name, timeout, command...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
    local rc=$?
    echo "$name exit $rc" >> "$OUT/steps.log"
    return $rc
}
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-host --no-shapes --extra none --steps 10 --warmup 2 $*"
step trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B || exit $?
step fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- $B || exit $?
step write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- $B || exit $?
step sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d "$OUT/sq" -o run --output-format csv -- $B || exit $?
step sq2 600 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/sq2" -o run --output-format csv -- $B || exit $?
step tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/tcc" -o run --output-format csv -- $B || exit $?
step ta 600 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum -d "$OUT/ta" -o run --output-format csv -- $B || exit $?
