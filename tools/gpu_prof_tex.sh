#!/bin/bash
# Texture-path PMC passes (TA busy/stalls, TCP->TCC latency, UTCL1 translation)
# for one bench config.  usage: gpu_prof_tex.sh TAG [bench args...]
R="$GRAFT_REPO_ROOT"; TAG=$1; shift
OUT="$R/gpurun_out/tex_$TAG"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-host --steps 6 --warmup 2 $*"
step() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; return $rc; }
step ta rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum -d "$OUT/ta" -o run --output-format csv -- $B || exit $?
step tcp rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum -d "$OUT/tcp" -o run --output-format csv -- $B || exit $?
step utcl rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_SERIALIZATION_STALL_sum -d "$OUT/utcl" -o run --output-format csv -- $B || exit $?
step grbm rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_TA_BUSY -d "$OUT/grbm" -o run --output-format csv -- $B || exit $?
