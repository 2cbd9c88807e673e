#!/bin/bash
# the part-wise (sharded) one-call evaluation: parity tests, per-part timing, the 2-rank bench path
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/part
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    tests/test_auc_cells_gpu.py -k "auc or compact or sorted" -m gpu > gpurun_out/part/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/probe_eval_part.py 30 > gpurun_out/part/probe.jsonl 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_gpu.py -m gpu \
    > gpurun_out/part/bench_tests.log 2>&1 || exit 1
