#!/bin/bash
# round 5: the gather-free two-step build (count from the slots), the check word without spill or
# per-wave atomics: AUC suites + the per-rank probe + its kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_two_step_gpu.py tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_auc.log 2>&1
rc=$?; echo "auc tests rc=$rc"; tail -4 $O/pytest_auc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 50 > $O/two_step.jsonl 2> $O/two_step.err || exit $?
cat $O/two_step.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace2 -o two_step -- python3 scripts/probe_two_step.py 20 --trace > $O/two_step_trace.log 2>&1 || exit $?
exit $rc
