#!/bin/bash
# Round 4: C5 fine-slot knob sweep, second pass (port bits x gain), and C3
# under the same knobs.  usage: gpu_r4v.sh TAG
R="$GRAFT_REPO_ROOT"; T=$1; OUT="$R/gpurun_out/$T"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 600 python tools/ab_env.py c5 5 base=NFFACL_AB:0 p5=NFFACL_TUNE_FINE_P:5 \
    p5g70=NFFACL_TUNE_FINE_P:5,NFFACL_TUNE_FINE_G:70 g70=NFFACL_TUNE_FINE_G:70 \
    p5g70m64=NFFACL_TUNE_FINE_P:5,NFFACL_TUNE_FINE_G:70,NFFACL_TUNE_FINE_MIN:64 \
    > "$OUT/ab_c5_fine_sweep2.json" 2> "$OUT/ab_c5.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c5_fine_sweep2.json"
timeout -k 10 600 python tools/ab_env.py c3 4 base=NFFACL_AB:0 p5g70=NFFACL_TUNE_FINE_P:5,NFFACL_TUNE_FINE_G:70 \
    > "$OUT/ab_c3_fine.json" 2> "$OUT/ab_c3.err" || exit 1
python -c "import json,sys;d=json.load(open(sys.argv[1]));print({k:(round(v['median_ms'],4),v['bit_exact_vs_first']) for k,v in d['variants'].items()})" "$OUT/ab_c3_fine.json"
