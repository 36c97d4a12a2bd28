#!/bin/bash
# Parity (whole -m gpu suite) on the working tree, then alternating-process
# A/B of the working library against a baseline build (build_prev/) on C2,
# C3, C5, then the C2 load modes in one process.  usage: gpu_r3n.sh TAG BASELIB
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$1"; BASE=$2; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.out" 2>&1 || { echo "pytest failed"; exit 1; }
for rep in 1 2; do for cfg in c2 c3 c5; do for lib in build_prev/$BASE libnffacl; do
  NFFACL_LIB=$R/nff-go_amd/$lib.so timeout -k 10 300 python tools/ab_env.py $cfg 4 d=NFFACL_AB:0 \
      > "$OUT/${cfg}_$(basename $lib)_$rep.json" 2>> "$OUT/err.log" || exit 1
done; done; done
[ -n "$MODES" ] || exit 0
timeout -k 10 300 python tools/ab_env.py c2 6 m4=NFFACL_TUNE_COAL:4 m4b768=NFFACL_TUNE_COAL:4,NFFACL_TUNE_BLOCK:768 \
    m5b768=NFFACL_TUNE_COAL:5,NFFACL_TUNE_BLOCK:768 m6=NFFACL_TUNE_COAL:6 \
    m7b768=NFFACL_TUNE_COAL:7,NFFACL_TUNE_BLOCK:768 > "$OUT/c2_modes.json" 2>> "$OUT/err.log" || exit 1
