#!/bin/bash
# Scalar-call sweep at 1 and 32 callers with the process pinned (taskset) to
# each NUMA node's CPUs in turn (first-touch puts the mailboxes there too), to
# see whether the consumer's bimodal poll / group times follow the node.
# usage: gpu_svc_numa.sh TAG
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/svcnuma_$1"; mkdir -p "$OUT"; cd "$R"
python tools/service_bench.py "$OUT/in" c2 || exit 1
for f in /sys/devices/system/node/node*/cpulist; do echo "$f $(cat $f)"; done > "$OUT/numa.txt"
cat /sys/class/drm/card*/device/numa_node >> "$OUT/numa.txt" 2>&1
grep -i cpus_allowed_list /proc/self/status >> "$OUT/numa.txt"
for rep in 1 2; do for nd in none /sys/devices/system/node/node0 /sys/devices/system/node/node1; do
  if [ "$nd" = none ]; then cpus=$(grep -i cpus_allowed_list /proc/self/status | awk '{print $2}'); node=none
  else [ -f $nd/cpulist ] || continue; cpus=$(cat $nd/cpulist); node=$(basename $nd); fi
  for t in 1 16 32; do
    timeout -k 10 60 taskset -c "$cpus" ./tools/service_bench "$OUT/in/rules.conf" "$OUT/in/slots.bin" "$OUT/in/expect.bin" $t 3 > "$OUT/r.json" 2>> "$OUT/err.log" || { echo "$node t $t failed" >> "$OUT/err.log"; continue; }
    echo "{\"node\": \"$node\", \"r\": $(cat $OUT/r.json)}" >> "$OUT/sweep.jsonl"
  done
done; done
rm -rf "$OUT/in"
