#!/bin/bash
# compaction with 1-bit masks: parity, kernel trace of the AUC micro, bench AUC legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02cm
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "auc or eval or sort or compact" tests/test_integration_gpu.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 scripts/micro_kernels.py \
    --which aucsort --reps 5 > $O/trace.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-train --no-surrogate --no-cpu-baseline > $O/bench_auc.json 2> $O/bench_auc.err || exit 1
