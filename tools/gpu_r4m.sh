#!/bin/bash
# Round 4: burst consumer, sequential polls (header-only vs whole mailbox,
# NFFACL_TUNE_SVC_FULLPOLL) with the vectorised host packing; C5 rounds per
# window 3 / 4 / 5 (NFFACL_EXP_R4 builds); two-stage flat entries (two.so) A/B + parity.  usage: gpu_r4m.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_service_burst.py tests/test_service.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.out" 2>&1 || { tail -30 "$OUT/pytest.out"; exit 1; }
tail -1 "$OUT/pytest.out"
for fp in 0 1; do
  NFFACL_TUNE_SVC_FULLPOLL=$fp NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5,burst:32:32:1.5,scalar:1:0:1.0,scalar:32:0:1.0" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/bench_shapes_fp$fp.json" 2> "$OUT/bench_shapes_fp$fp.err" || exit 1
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('fp$fp',{k:(v['mpps'],v['lat_us_p50'],v['lat_us_p99'],v['consumer_poll_us'],v['consumer_group_us'],v['wrong']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/bench_shapes_fp$fp.json"
done
NOTEST=1 CFGS="c5 c3" ROUNDS=3 bash tools/gpu_libab.sh "$T/lib" nff-go_amd/build_exp/base.so nff-go_amd/libnffacl.so \
    nff-go_amd/build_exp/r3.so nff-go_amd/build_exp/r5.so || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider -k "hybrid or c5 or c3" > "$OUT/pytest_two.out" 2>&1 \
    || { tail -30 "$OUT/pytest_two.out"; exit 1; }
tail -1 "$OUT/pytest_two.out"
timeout -k 10 300 python tools/svc_overlap.py 4 > "$OUT/svc_overlap.json" 2> "$OUT/svc_overlap.err" || { tail -5 "$OUT/svc_overlap.err"; exit 1; }
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:d[k] for k in ('alone_ms','armed_ms','after_ms','slowdown_armed','calls_during')})" "$OUT/svc_overlap.json"
