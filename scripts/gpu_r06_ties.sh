#!/bin/bash
# round 6: the distinct-key index of tie-heavy tables -- its GPU tests and the AUC suites around it,
# the one-call timings per score distribution, and a kernel trace of the bf16-rounded 2^27 case
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r06ties8}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_auc_ties_gpu.py tests/test_auc_cells_gpu.py tests/test_kernels_gpu.py tests/test_two_step_gpu.py > $O/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/probe_eval_ties.py 10 > $O/ties.jsonl 2> $O/ties.err &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o ties -- \
    python3 scripts/probe_eval_ties.py 5 --only bf16 27 > $O/trace_log.txt 2>&1 &&
python3 scripts/kernels_by_grid.py $O/trace $O/kernels_by_grid.json &&
timeout -k 10 180 python -u scripts/probe_dk_query.py 20 > $O/dk_u.jsonl 2> $O/dk_u.err && echo done
