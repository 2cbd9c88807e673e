#!/bin/bash
# round 6: the slotted count pass with its key, header and histogram loads issued together
#  -- the two-step GPU tests, then the per-rank probe interleaving the product
# library with the previous commit's build (tuning/libdauc_base.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06cnt
mkdir -p $O
scripts/gpu_step.sh r06cnt/pytest_two_step 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_two_step_gpu.py; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 40 --base=tuning/libdauc_base.so > $O/probe_base.jsonl 2> $O/probe_base.err; rc=$?
echo "probe rc=$rc"; cat $O/probe_base.jsonl; tail -3 $O/probe_base.err
exit $rc
