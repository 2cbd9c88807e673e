#!/bin/bash
# round 3: the GPU suite on the new eval ABI / tail kernels, the tail stamps, the loss A/B, the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh pytest_gpu 540 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh stamps5 120 python -u scripts/probe_tail_stamps.py 15 5; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh stamps7 120 python -u scripts/probe_tail_stamps.py 15 7; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ab_sur 180 python -u scripts/ab_surrogate.py 3 100 0,3,4,6,8,9; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench 480 python -u bench.py; rc=$?
exit $rc
