#!/bin/bash
# Parity subset (PYK: pytest -k expression; NOTEST=1 skips it), then a
# one-process interleaved A/B of NFFACL_TUNE_* variants (tools/ab_env.py)
# per config, every variant bit-exact against the first.
# usage: gpu_ab.sh TAG ROUNDS "CFG..." NAME=VAR:VAL[,VAR:VAL] ...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$1"; ROUNDS=$2; CFGS=$3; shift 3; mkdir -p "$OUT"; cd "$R"
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q ${PYK:+-k "$PYK"} --timeout 300 --timeout-method thread \
      -p no:cacheprovider > "$OUT/pytest.out" 2>&1 || { echo "pytest failed"; tail -40 "$OUT/pytest.out"; exit 1; }
  tail -2 "$OUT/pytest.out"
fi
for cfg in $CFGS; do
  timeout -k 10 300 python tools/ab_env.py "$cfg" "$ROUNDS" "$@" > "$OUT/ab_$cfg.json" 2> "$OUT/ab_$cfg.err" \
      || { echo "ab $cfg failed"; tail -20 "$OUT/ab_$cfg.err"; exit 1; }
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[2], {k:(round(v['median_ms'],4), v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_$cfg.json" "$cfg"
done
