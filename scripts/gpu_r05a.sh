#!/bin/bash
# round 5: the two-step sharded evaluation's new checks + the RCCL rehearsal, then the AUC suites
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
export DAUC_BENCH_RECORD_DIR=$O
timeout -k 10 600 python -u -m pytest tests/test_two_step_gpu.py tests/test_rccl_rehearsal_gpu.py -v --timeout 560 --timeout-method thread > $O/pytest_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -15 $O/pytest_new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest_auc.log 2>&1
rc2=$?; echo "auc suites rc=$rc2"; tail -8 $O/pytest_auc.log
exit $(( rc > rc2 ? rc : rc2 ))
