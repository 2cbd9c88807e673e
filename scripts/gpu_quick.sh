#!/bin/bash
# parity tests + kernel micro-benchmarks
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh micro 300 python -u scripts/micro_kernels.py --which ${MICRO:-update,surrogate}; rc=$?
exit $rc
