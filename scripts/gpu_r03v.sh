#!/bin/bash
# round 3: the compactions with their label loads batched in straight-line code (DAUC_COMPACT_BATCH
# = 8, the default now; cb0 = round 2's per-group branches) -- the GPU suites that compact, then
# per-kernel times of both builds (one-call evaluation and the two-pass compaction of probe_query)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/cb
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py -x -v --timeout 200 --timeout-method thread > $O/product_tests.log 2>&1 || exit $?
for v in tuning cb0; do
  export DAUC_LIB=tuning/libdauc_$v.so
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt_$v -- python3 scripts/ab_eval.py 10 $v > $O/log_kt_$v.txt 2>&1 || exit 1
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o pq_$v -- python3 scripts/probe_query.py 27 0.001 3 > $O/log_pq_$v.txt 2>&1 || exit 1
done
