#!/bin/bash
# evaluation host path trimmed: parity, then the bench's AUC legs (wall clock per evaluation)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02ew
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "auc or eval or sort" tests/test_integration_gpu.py tests/test_main_gpu.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-train --no-surrogate --no-cpu-baseline >> $O/bench_auc.jsonl 2>> $O/bench_auc.err || exit 1
done
