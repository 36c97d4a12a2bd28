#!/bin/bash
# Round 4: flat-walk cost breakdown on C5 (timing probes, verdicts wrong):
# NFFACL_EXP_FLAT 1 own fields (no ds_bpermute), 2 no rule test, 4 no IPv6
# second stage, 8 no LDS atomics; NFFACL_EXP_ENTLOAD 2 no entry loads.
# usage: gpu_r4h.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; cd "$R"
NOTEST=1 CFGS="c5" ROUNDS=3 bash tools/gpu_libab.sh "$T/lib" nff-go_amd/libnffacl.so nff-go_amd/build_exp/fl1.so \
    nff-go_amd/build_exp/fl2.so nff-go_amd/build_exp/fl4.so nff-go_amd/build_exp/fl8.so nff-go_amd/build_exp/ent2.so
