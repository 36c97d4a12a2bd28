#!/bin/bash
# Round 4: C5 fine-slot knob sweep (NFFACL_TUNE_FINE_*), env A/B in one
# process, every variant bit-exact against the first.  usage: gpu_r4u.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python tools/ab_env.py c5 4 base=NFFACL_AB:0 g30=NFFACL_TUNE_FINE_G:30 g70=NFFACL_TUNE_FINE_G:70 \
    p5=NFFACL_TUNE_FINE_P:5 p6=NFFACL_TUNE_FINE_P:6 a10=NFFACL_TUNE_FINE_A:10 min64=NFFACL_TUNE_FINE_MIN:64 \
    s15=NFFACL_TUNE_FINE_SLOTS:15 > "$OUT/ab_c5_fine_sweep.json" 2> "$OUT/ab_c5.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c5_fine_sweep.json"
