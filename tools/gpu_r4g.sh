#!/bin/bash
# Round 4: is the flat walk bound by the vector-memory pipeline?  Library A/B
# of the entry-load probes (NFFACL_EXP_ENTLOAD 1: one 16-byte load per
# candidate, 2: none; timing only, verdicts wrong) on C5 and C3, and the TA /
# TCP counters of the C5 kernel.  usage: gpu_r4g.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
NOTEST=1 CFGS="c5 c3" ROUNDS=3 bash tools/gpu_libab.sh "$T/lib" nff-go_amd/libnffacl.so nff-go_amd/build_exp/ent1.so \
    nff-go_amd/build_exp/ent2.so || exit 1
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-host --extra none --steps 10 --warmup 2 --config c5"
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum \
    -d "$OUT/pmc_ta" -o run --output-format csv -- $B > "$OUT/pmc_ta.out" 2> "$OUT/pmc_ta.err" || exit 1
python3 "$R/tools/pmc_sq.py" "$OUT/pmc_ta" k_indexed
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES \
    -d "$OUT/pmc_sq" -o run --output-format csv -- $B > "$OUT/pmc_sq.out" 2> "$OUT/pmc_sq.err" || exit 1
python3 "$R/tools/pmc_sq.py" "$OUT/pmc_sq" k_indexed
