#!/bin/bash
# round 4: slot histograms (no histogram pass in the query part) and records counted in place:
# the part probe and the two-step / AUC tests
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04o
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_slots_gpu.py tests/test_auc_cells_gpu.py -q --timeout 300 --timeout-method thread > $D/pytest_auc.log 2>&1
rc=$?
echo "auc tests rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/probe_eval_part.py 20 > $D/eval_part_probe.jsonl 2> $D/eval_part_probe.err || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/probe -o run -- python3 $GRAFT_REPO_ROOT/scripts/probe_eval_part.py 5 > $GRAFT_REPO_ROOT/$D/probe_trace.log 2>&1 || exit 1
