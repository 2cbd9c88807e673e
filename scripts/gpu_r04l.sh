#!/bin/bash
# round 4: the query pass's counts reduced through 8 group partials (no 256-deep atomic queue at
# its end): AUC tests, the query intercept trace and the part probe
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04l
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_slots_gpu.py tests/test_auc_cells_gpu.py -q --timeout 300 --timeout-method thread > $D/pytest_auc.log 2>&1
rc=$?
echo "auc tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/probe_query_intercept.py 10 > $GRAFT_REPO_ROOT/$D/trace.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python -u scripts/probe_eval_part.py 20 > $D/eval_part_probe.jsonl 2> $D/eval_part_probe.err || exit 1
