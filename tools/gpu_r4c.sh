#!/bin/bash
# Round 4: new tests (C++ mirror bursts, full-size C3, services), fine 2-D slot
# parity + A/B on C5/C3, burst-shape sweep on C2.  usage: gpu_r4c.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -k "cpp or full_size_c3 or service" --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest_new.out" 2>&1 || { tail -30 "$OUT/pytest_new.out"; exit 1; }
tail -1 "$OUT/pytest_new.out"
NFFACL_TUNE_FINE_A=8 NFFACL_TUNE_FINE_P=4 NFFACL_TUNE_FINE_MIN=16 NFFACL_TUNE_DIR_PER_RULE=16 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    -k "hybrid or c5 or c3 or test_service" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_fine.out" 2>&1 || { tail -30 "$OUT/pytest_fine.out"; exit 1; }
tail -1 "$OUT/pytest_fine.out"
for c in c5 c3; do
  if [ $c = c5 ]; then V="fine84=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:4 fine83=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:3"
  else V="fine=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_MIN:16,NFFACL_TUNE_DIR_PER_RULE:16 dir16=NFFACL_TUNE_DIR_PER_RULE:16"; fi
  timeout -k 10 600 python tools/ab_env.py $c 4 base=NFFACL_AB:0 $V > "$OUT/ab_$c.json" 2> "$OUT/ab_$c.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], {k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_$c.json"
done
NOTEST=1 CFGS="c5 c3" ROUNDS=3 bash tools/gpu_libab.sh "$T/saddr" nff-go_amd/libnffacl.so nff-go_amd/build_exp/saddr0.so || exit 1
NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:4:32:1.0,burst:16:32:1.5,burst:32:32:1.5,scalar:32:0:1.0" \
  timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
    > "$OUT/bench_shapes.json" 2> "$OUT/bench_shapes.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(json.dumps(d.get('call_shapes')))" "$OUT/bench_shapes.json"
