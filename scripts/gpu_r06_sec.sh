#!/bin/bash
# round 6: the carried secondary window (query_ci_kernel's SEC): the exact-AUC GPU tests on the
# product build, then scripts/probe_query_sec.py's interleaved A/B on the tuning build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06sec2
mkdir -p $O
timeout -k 10 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_two_step_gpu.py tests/test_auc_cells_gpu.py > $O/tests.log 2>&1 &&
timeout -k 10 240 python -u scripts/probe_query_sec.py 50 > $O/ab.jsonl 2> $O/ab.err &&
echo done
