#!/bin/bash
# Round 4: C2 LDS-conflict A/B (library builds) + fine 2-D slot parity and
# A/B on C5/C3 + call-shape record (C2).  usage: gpu_r4b.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
NOTEST=1 PMC=1 CFGS=c2 bash tools/gpu_libab.sh "$T/lds" nff-go_amd/libnffacl.so nff-go_amd/build_exp/lds0.so \
    nff-go_amd/build_exp/lds2.so || exit 1
NFFACL_TUNE_FINE_A=8 NFFACL_TUNE_FINE_P=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q \
    -k "hybrid or c5 or c3 or service or full_size" --timeout 120 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_fine.out" 2>&1 || { tail -30 "$OUT/pytest_fine.out"; exit 1; }
tail -2 "$OUT/pytest_fine.out"
for c in c5 c3; do
  timeout -k 10 600 python tools/ab_env.py $c 4 base=NFFACL_AB:0 fine84=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:4 \
      fine83=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:3 > "$OUT/ab_$c.json" 2> "$OUT/ab_$c.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], {k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_$c.json"
done
timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
    > "$OUT/bench_shapes.json" 2> "$OUT/bench_shapes.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(json.dumps(d.get('call_shapes')))" "$OUT/bench_shapes.json"
