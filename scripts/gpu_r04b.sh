#!/bin/bash
# round 4: the range-bucketed exact AUC: AUC GPU tests, eval timing, kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
D=gpurun_out/r04b
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "auc or sort or split or compact" > $D/pytest_auc.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_eval.py 20 bucket > $D/ab_eval.jsonl 2> $D/ab_eval.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/ab_eval.py 5 bucket > $GRAFT_REPO_ROOT/$D/prof.log 2>&1
