#!/bin/bash
# surrogate kernel: parity tests, then the geometry sweep (scripts/micro_kernels.py)
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_sur 300 python -u -m pytest tests/test_kernels_gpu.py -k surrogate -x -v --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh micro_sur 300 python -u scripts/micro_kernels.py --which surrogate --sur-variants 0,1,2,3,4,5,6,7 --reps 20; rc=$?
exit $rc
