#!/bin/bash
# Parity (whole -m gpu suite unless NOTEST=1, or the -k subset in PYK) on the
# working tree, then an alternating-process A/B of library builds (paths
# relative to the repo, .so included) on CFGS (default c2), then, with PMC=1,
# one rocprofv3 counter pass per library (SQ LDS / VALU counters of the C2
# bench kernel).  usage: gpu_libab.sh TAG LIB...
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/$1"; shift; mkdir -p "$OUT"; cd "$R"
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q ${PYK:+-k "$PYK"} --timeout 120 --timeout-method thread \
      -p no:cacheprovider > "$OUT/pytest.out" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.out"; exit 1; }
  tail -3 "$OUT/pytest.out"
fi
for rep in 1 2; do for cfg in ${CFGS:-c2}; do for lib in "$@"; do
  NFFACL_LIB=$R/$lib timeout -k 10 300 python tools/ab_env.py $cfg ${ROUNDS:-4} d=NFFACL_AB:0 \
      > "$OUT/${cfg}_$(dirname $lib | tr / _)_$rep.json" 2>> "$OUT/err.log" || { echo "ab $cfg $lib failed"; exit 1; }
  echo "$cfg $lib $rep $(python -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['variants']['d']['median_ms'])" "$OUT/${cfg}_$(dirname $lib | tr / _)_$rep.json")"
done; done; done
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  for cfg in ${CFGS:-c2}; do for lib in "$@"; do
    d="$OUT/pmc_${cfg}_$(basename $lib .so)"
    NFFACL_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
        SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU -d "$d" -o run --output-format csv -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-host --extra none --steps 10 --warmup 2 --config $cfg \
        > "$d.out" 2> "$d.err" || { echo "pmc $cfg $lib failed"; exit 1; }
    python3 "$R/tools/pmc_sq.py" "$d" k_indexed
  done; done
fi
