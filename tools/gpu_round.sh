#!/bin/bash
# One GPU call: the whole -m gpu suite, then tools/gpu_exp.sh (service sweep
# per variant + library A/B), then the host-inclusive modes.
# usage: gpu_round.sh TAG "CFGS" "LIB..." "VAR=VAL"...
R="$GRAFT_REPO_ROOT"; TAG=$1; cd "$R"; OUT="$R/gpurun_out/round_$TAG"; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 150 --timeout-method thread -p no:cacheprovider tests \
    > "$OUT/pytest.out" 2>&1 || { echo "pytest failed" >> "$OUT/steps.log"; exit 1; }
echo "pytest ok" >> "$OUT/steps.log"
bash tools/gpu_exp.sh "$@" || { echo "exp failed" >> "$OUT/steps.log"; exit 1; }
echo "exp ok" >> "$OUT/steps.log"
timeout -k 10 300 python tools/host_modes.py c2 23 > "$OUT/host_modes.json" 2> "$OUT/host_modes.err" || exit 1
echo "host ok" >> "$OUT/steps.log"
