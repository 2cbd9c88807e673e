#!/bin/bash
# round 3, first check: the new configs[2] 8-rank test, the GPU suite, the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh configs2 700 python -u -m pytest tests/test_configs2_gpu.py -x -v --timeout 680 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh pytest_gpu 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread --deselect tests/test_configs2_gpu.py::test_configs2_resnet50_8ranks_period_sweep; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench 420 python -u bench.py; rc=$?
exit $rc
