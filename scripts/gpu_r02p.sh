#!/bin/bash
# one-pass (decoupled look-back) positive compaction: parity, AUC timings and kernel trace
set -o pipefail
mkdir -p gpurun_out/r02r
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "compact or auc or sorted or extreme" tests/test_integration_gpu.py > gpurun_out/r02r/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 > gpurun_out/r02r/micro.jsonl 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02r/trace -o run -- python3 scripts/micro_kernels.py \
    --which aucsort --reps 5 > gpurun_out/r02r/trace.log 2>&1 || exit 1
