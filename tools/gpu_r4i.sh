#!/bin/bash
# Round 4: C5 walk floor (NFFACL_EXP_FLAT 16: no candidate windows at all;
# ENTLOAD 2: windows without entry loads) and the PCIe read probe of the
# burst mailbox poll.  usage: gpu_r4i.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
NOTEST=1 CFGS="c5" ROUNDS=3 bash tools/gpu_libab.sh "$T/lib" nff-go_amd/libnffacl.so nff-go_amd/build_exp/fl16.so \
    nff-go_amd/build_exp/ent2.so || exit 1
timeout -k 10 300 tools/pcie_probe > "$OUT/pcie_probe.jsonl" 2> "$OUT/pcie_probe.err" || exit 1
wc -l "$OUT/pcie_probe.jsonl"
