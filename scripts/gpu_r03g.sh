#!/bin/bash
# round 3: eval-forward determinism probe; loss-kernel tail variants (extra reducer workgroups) A/B + stamps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh det 180 python -u scripts/probe_eval_determinism.py 48; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ab_sur 240 python -u scripts/ab_surrogate.py 3 100 0,3,4,10,11,12,13,15,16; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh stamps14 120 python -u scripts/probe_tail_stamps.py 15 14; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh stamps5 120 python -u scripts/probe_tail_stamps.py 15 5; rc=$?
exit $rc
