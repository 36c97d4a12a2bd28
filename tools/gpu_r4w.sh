#!/bin/bash
# Round 4: where the burst call's answer -> next-request gap goes
# (NFFACL_EXP_SVCSTAT builds: 3 = gap statistic + no classification,
# 5 = gap statistic + stop word read every 64th pass).  usage: gpu_r4w.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
for v in ${VARIANTS:-svc3 svc5}; do
  NFFACL_LIB=$R/nff-go_amd/build_exp/$v.so NFFACL_BENCH_SHAPES="burst:1:32:1.0,burst:16:32:1.5" \
    timeout -k 10 300 python bench.py --extra none --no-cpu-baseline --no-host --steps 5 --warmup 2 \
      > "$OUT/$v.json" 2> "$OUT/$v.err"
  rc=$?; [ $rc -le 1 ] || exit 1  # (svc3 answers without classifying: bench exits 1 on its wrong verdicts)
  python -c "import json,sys;d=json.load(open(sys.argv[1]))['call_shapes']['c2'];print('$v',{k:(v['mpps'],v['lat_us_p50'],v['consumer_poll_us'],v['consumer_group_us']) for k,v in d.items() if isinstance(v,dict)})" "$OUT/$v.json"
done
