#!/bin/bash
# Round 4: C5 with two workgroups per CU (new default) vs one
# (NFFACL_TUNE_PER_CU=1), parity subset, and beside busy consumers.  usage: gpu_r4ee.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider -k "c5 or hybrid" > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
timeout -k 10 600 python tools/ab_env.py c5 5 new=NFFACL_AB:0 pc1=NFFACL_TUNE_PER_CU:1 > "$OUT/ab_c5_pc.json" 2> "$OUT/ab_c5.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c5_pc.json"
timeout -k 10 300 python tools/svc_overlap.py 4 > "$OUT/svc_overlap.json" 2> "$OUT/svc_overlap.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:d[k] for k in ('alone_ms','armed_ms','slowdown_armed')})" "$OUT/svc_overlap.json"
