#!/bin/bash
# query kernel with the 4-VALU tree step: parity, timings, then a kernel trace
set -o pipefail
mkdir -p gpurun_out/r02d
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "compact or nonfinite or extreme or sorted_counts or auc or radix" > gpurun_out/r02d/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 > gpurun_out/r02d/micro.jsonl 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02d/trace -o run -- python3 scripts/probe_query.py 27 0.001 5 \
    > gpurun_out/r02d/trace.log 2>&1
