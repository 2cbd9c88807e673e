#!/bin/bash
# round 6: the slotted two-step build -- the AUC GPU tests, then the A/B per-rank
# probe of step 2's two forms (tuning build), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06slot
mkdir -p $O
scripts/gpu_step.sh r06slot/pytest_auc 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_two_step_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py \
    tests/test_kernels_gpu.py -k "auc or eval or two_step or count or split or pair or sort"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 30 --ab > $O/probe_ab.jsonl 2> $O/probe_ab.err; rc=$?
echo "probe rc=$rc"; cat $O/probe_ab.jsonl
exit $rc
