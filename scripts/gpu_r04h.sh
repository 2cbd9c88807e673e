#!/bin/bash
# round 4: the compaction stages the positives' scores in LDS while its reservation is in flight:
# the AUC / count-index / slot tests, the part probe
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04h
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_slots_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py -q --timeout 300 --timeout-method thread > $D/pytest_auc.log 2>&1
rc=$?
echo "auc tests rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/probe_eval_part.py 20 > $D/eval_part_probe.jsonl 2> $D/eval_part_probe.err || exit 1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/prof_eval.py 27 0.001 10 > $GRAFT_REPO_ROOT/$D/prof.log 2>&1 || exit 1
