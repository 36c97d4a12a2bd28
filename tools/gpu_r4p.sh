#!/bin/bash
# Round 4: mailbox round trip with the consumer's extras one at a time
# (tools/mailbox_probe.hip), pinned to a CPU of the GPU's node.  usage: gpu_r4p.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
NODE=$(python -c "import sys; sys.path.insert(0,'nff-go_amd'); import nffacl; print(nffacl.device_numa_node(0))")
CPU=$(python -c "
import os,sys
n=int(sys.argv[1]); allowed=os.sched_getaffinity(0)
try:
    s=open(f'/sys/devices/system/node/node{n}/cpulist').read().strip()
    cpus=[c for part in s.split(',') for c in (range(int(part.split('-')[0]),int(part.split('-')[-1])+1))]
    cpus=[c for c in cpus if c in allowed]
    print(cpus[0] if cpus else min(allowed))
except Exception: print(min(allowed))" "$NODE")
echo "node $NODE cpu $CPU"
timeout -k 10 120 tools/mailbox_probe "$CPU" > "$OUT/mailbox_variants.jsonl" 2>&1 || { cat "$OUT/mailbox_variants.jsonl"; exit 1; }
cat "$OUT/mailbox_variants.jsonl"
