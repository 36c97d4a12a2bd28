#!/bin/bash
# Profile the default (AUTO) kernels of C2, C3 and C5.  usage: gpu_prof3.sh TAG
R="$GRAFT_REPO_ROOT"; TAG=$1
for cfg in c3 c5 c2; do
  bash "$R/tools/gpu_prof.sh" "${TAG}_$cfg" --config $cfg || exit $?
done
