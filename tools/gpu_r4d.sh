#!/bin/bash
# Round 4: burst sub-mailboxes (tests + sweep), C5 fine-slot shapes x load
# modes, C3 directory resolution.  usage: gpu_r4d.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "burst or cpp or test_service" --timeout 300 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5,burst:32:32:1.5" \
  timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
    > "$OUT/bench_shapes.json" 2> "$OUT/bench_shapes.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(json.dumps(d.get('call_shapes')))" "$OUT/bench_shapes.json"
F83=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:3
F84=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:4,NFFACL_TUNE_FINE_SLOTS:3
timeout -k 10 600 python tools/ab_env.py c5 4 base=NFFACL_AB:0 f83=$F83 f83m4=$F83,NFFACL_TUNE_COAL:4 \
    f84s=$F84 f84sm4=$F84,NFFACL_TUNE_COAL:4 > "$OUT/ab_c5.json" 2> "$OUT/ab_c5.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], {k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c5.json"
timeout -k 10 600 python tools/ab_env.py c3 4 base=NFFACL_AB:0 d16=NFFACL_TUNE_DIR_PER_RULE:16 \
    d32=NFFACL_TUNE_DIR_PER_RULE:32 d8=NFFACL_TUNE_DIR_PER_RULE:8 > "$OUT/ab_c3.json" 2> "$OUT/ab_c3.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], {k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c3.json"
