#!/bin/bash
# 1x1-conv / skip-branch parity tests, then a short bench of the training step (no AUC / CPU legs)
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_skip 300 python -u -m pytest tests/test_conv1x1_gpu.py tests/test_maxpool_gpu.py tests/test_coda_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench_train 400 python -u bench.py --steps 20 --warmup 5 --no-auc --no-surrogate --no-cpu-baseline; rc=$?
exit $rc
