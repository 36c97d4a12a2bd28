#!/bin/bash
# C3 occupancy experiment (frames kernels compiled for 6 waves per SIMD, two
# 768-thread workgroups per CU over smaller directories), the scalar-call
# sweep, then the round's rocprofv3 traces + PMC of C3, C5, C2.
R="$GRAFT_REPO_ROOT"; cd "$R"; OUT="$R/gpurun_out/r3m"; mkdir -p "$OUT"
V="base= occ56=NFFACL_TUNE_DIR_KB:56,NFFACL_TUNE_BLOCK:768,NFFACL_TUNE_PER_CU:2 occ64=NFFACL_TUNE_DIR_KB:64,NFFACL_TUNE_BLOCK:768,NFFACL_TUNE_PER_CU:2"
for lib in libnffacl_r3i libnffacl_wpe6; do
  NFFACL_LIB=$R/nff-go_amd/build_prev/$lib.so timeout -k 10 300 python tools/ab_env.py c3 3 $V > "$OUT/c3_$lib.json" 2> "$OUT/c3_$lib.err" || exit 1
  echo "ab $lib ok" >> "$OUT/steps.log"
done
bash tools/gpu_svc_sweep.sh r3m c2 "NFFACL_TUNE_SVC_SLEEP_NS=-1" "NFFACL_TUNE_SVC_SLEEP_NS=0" || exit 1
echo "sweep ok" >> "$OUT/steps.log"
bash tools/gpu_prof3.sh r3 || exit 1
echo "prof ok" >> "$OUT/steps.log"
