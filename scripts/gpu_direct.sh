#!/bin/bash
# the direct count-index build in the one-call evaluation: parity, timing, kernel trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/direct
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    tests/test_auc_cells_gpu.py tests/test_integration_gpu.py -k "auc or compact or sorted or eval" -m gpu \
    > gpurun_out/direct/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/probe_eval_part.py 30 > gpurun_out/direct/probe.jsonl 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/direct/trace -o run -- \
    python3 scripts/probe_eval_part.py 5 > gpurun_out/direct/trace.log 2>&1 || exit 1
