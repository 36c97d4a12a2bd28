#!/bin/bash
# L2 ACL parity (GPU), then the current library against nff-go_amd/libnffacl_prev.so
# (a build of the previous variant), alternating processes on one box.
# usage: gpu_l2ab.sh TAG
TAG=$1; R="$GRAFT_REPO_ROOT"; cd "$R"
OUT="$R/gpurun_out/l2ab_$TAG"; mkdir -p "$OUT"
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name exit $rc" >> "$OUT/steps.log"; [ $rc -eq 0 ] || exit $rc; }
step pytest bash -c "timeout -k 10 600 python -u -m pytest tests/test_l2.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest.out 2>&1"
for i in 1 2; do
  step "prev$i" bash -c "NFFACL_LIB=$R/nff-go_amd/libnffacl_prev.so timeout -k 10 300 python tools/ab_env.py l2 4 x= > $OUT/prev$i.json 2> $OUT/prev$i.err"
  step "new$i" bash -c "timeout -k 10 300 python tools/ab_env.py l2 4 x= > $OUT/new$i.json 2> $OUT/new$i.err"
done
