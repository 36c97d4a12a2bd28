#!/bin/bash
# Parity (whole -m gpu suite, unless NOTEST=1) on the working tree, then an
# alternating-process A/B of library builds (paths under nff-go_amd/ without
# .so; the working library is `libnffacl`) on CFGS (default c2 c3 c5).
# usage: gpu_r3n.sh TAG LIB...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$1"; shift; mkdir -p "$OUT"; cd "$R"
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.out" 2>&1 || { echo "pytest failed"; exit 1; }
for rep in 1 2; do for cfg in ${CFGS:-c2 c3 c5}; do for lib in "$@"; do
  NFFACL_LIB=$R/nff-go_amd/$lib.so timeout -k 10 300 python tools/ab_env.py $cfg 4 d=NFFACL_AB:0 \
      > "$OUT/${cfg}_$(basename $lib)_$rep.json" 2>> "$OUT/err.log" || exit 1
done; done; done
