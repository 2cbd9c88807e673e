#!/bin/bash
# round 6: the slotted two-step query counts #(== x) only in groups where some lane has a tie
# (the compares or-ed into a lane mask) -- the AUC GPU tests, then the per-rank probe interleaving
# the product library with the zeroing-launch commit (tuning/libdauc_zero2.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06tie
mkdir -p $O
scripts/gpu_step.sh r06tie/pytest_auc 480 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_two_step_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py tests/test_auc_fuzz_gpu.py tests/test_auc_ties_gpu.py \
    tests/test_kernels_gpu.py -k "auc or eval or two_step or count or split or pair or sort or fuzz"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 40 --base=tuning/libdauc_zero2.so > $O/probe_base.jsonl 2> $O/probe_base.err; rc=$?
echo "probe rc=$rc"; tail -2 $O/probe_base.err
exit $rc
