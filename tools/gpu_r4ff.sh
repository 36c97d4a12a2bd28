#!/bin/bash
# Round 4: C5 fine-grid knob sweep around the 8 x 5 default.  usage: gpu_r4ff.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python tools/ab_env.py c5 5 base=NFFACL_AB:0 min128=NFFACL_TUNE_FINE_MIN:128 g60=NFFACL_TUNE_FINE_G:60 \
    s7=NFFACL_TUNE_FINE_SLOTS:7 a9=NFFACL_TUNE_FINE_A:9 > "$OUT/ab_c5_fine_sweep3.json" 2> "$OUT/ab_c5.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c5_fine_sweep3.json"
