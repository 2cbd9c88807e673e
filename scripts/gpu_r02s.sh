#!/bin/bash
# single-call evaluation (C orchestration): parity, then AUC timings and kernel trace
set -o pipefail
mkdir -p gpurun_out/r02w
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "compact or auc or sort or extreme or radix" tests/test_integration_gpu.py tests/test_main_gpu.py \
    > gpurun_out/r02w/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 > gpurun_out/r02w/micro.jsonl 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02w/trace -o run -- python3 scripts/micro_kernels.py \
    --which aucsort --reps 5 > gpurun_out/r02w/trace.log 2>&1 || exit 1
