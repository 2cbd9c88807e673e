#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_gpu 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
rm -f gpurun_out/sweep_sur.log
scripts/gpu_sweep_sur.sh; rc=$?; ok $rc || exit $rc
scripts/gpu_step.sh micro_pc 300 python -u scripts/micro_kernels.py --which paircount; rc=$?
exit $rc
