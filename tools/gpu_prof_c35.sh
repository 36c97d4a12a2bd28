#!/bin/bash
# rocprofv3 trace + PMC passes of the C3 and C5 benches (HYBRID flat-LDS).  usage: gpu_prof_c35.sh TAG
R="$GRAFT_REPO_ROOT"
bash "$R/tools/gpu_prof.sh" "${1}_c5" --config c5 || exit $?
bash "$R/tools/gpu_prof.sh" "${1}_c3" --config c3 || exit $?
