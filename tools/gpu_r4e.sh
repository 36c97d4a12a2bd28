#!/bin/bash
# Round 4: full GPU suite on the spill-free flat kernels, library A/B vs the
# previous commit, C5 fine-slot x load-mode A/B, burst sweep with and without
# streaming request stores.  usage: gpu_r4e.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
NOTEST=1 CFGS="c5 c3 c2" ROUNDS=3 bash tools/gpu_libab.sh "$T/lib" nff-go_amd/libnffacl.so nff-go_amd/build_exp/head.so || exit 1
F84=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:4,NFFACL_TUNE_FINE_SLOTS:3
F83=NFFACL_TUNE_FINE_A:8,NFFACL_TUNE_FINE_P:3
timeout -k 10 600 python tools/ab_env.py c5 4 base=NFFACL_AB:0 m4=NFFACL_TUNE_COAL:4 f84s=$F84 \
    f84sm4=$F84,NFFACL_TUNE_COAL:4 f83m4=$F83,NFFACL_TUNE_COAL:4 > "$OUT/ab_c5.json" 2> "$OUT/ab_c5.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], {k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c5.json"
for nt in 0 1; do
  NFFACL_TUNE_SVC_NT=$nt NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5,burst:32:32:1.5,scalar:1:0:1.0,scalar:32:0:1.0" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/bench_shapes_nt$nt.json" 2> "$OUT/bench_shapes_nt$nt.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('nt$nt', {k:(v['mpps'],v['lat_us_p50'],v['consumer_poll_us'],v['consumer_group_us']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/bench_shapes_nt$nt.json"
done
