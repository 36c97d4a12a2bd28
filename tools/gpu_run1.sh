#!/bin/bash
# First GPU session: parity tests, then the bench (only if the tests ended cleanly).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.log
rc=$?
echo "bench exit $rc" >> gpurun_out/bench.log
exit $rc
