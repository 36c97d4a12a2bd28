#!/bin/bash
# Round record: gpu_final.sh (parity suite, smoke, every config's bench line),
# then rocprofv3 kernel trace + PMC passes of the C2 headline and L2 benches.
# usage: gpu_record.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"
bash "$R/tools/gpu_final.sh" "$TAG" || exit $?
bash "$R/tools/gpu_prof.sh" "${TAG}_c2" || exit $?
bash "$R/tools/gpu_prof.sh" "${TAG}_l2" --config l2 || exit $?
