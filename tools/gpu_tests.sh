#!/bin/bash
# Full GPU test suite only.
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/tests_$1"; mkdir -p "$OUT"; cd "$R"
make -s -C tests/cpp > "$OUT/make.out" 2>&1
timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider --durations=15 > "$OUT/pytest.out" 2>&1
rc=$?; echo "pytest exit $rc" >> "$OUT/steps.log"; exit $rc
