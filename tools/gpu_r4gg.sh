#!/bin/bash
# Round 4: flat-LDS entry addresses from byte deltas (NFFACL_EXP_BDELTA=1
# build): HYBRID parity subset on that build, then library A/B on C5 / C3.
# usage: gpu_r4gg.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
NFFACL_LIB=$R/nff-go_amd/build_exp/bdelta.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "c5 or c3 or hybrid" > "$OUT/pytest.out" 2>&1 \
    || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
NOTEST=1 CFGS="c5 c3" ROUNDS=4 bash tools/gpu_libab.sh "$T/lib" nff-go_amd/libnffacl.so nff-go_amd/build_exp/bdelta.so || exit 1
