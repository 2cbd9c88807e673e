#!/bin/bash
# round 2: new AUC compaction / lockstep query and surrogate span variants: parity, then micro timings
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "compact or nonfinite or extreme or sorted_counts or chunked_variants or auc" > gpurun_out/r02a_tests.log 2>&1 &&
timeout -k 10 240 python -u scripts/micro_kernels.py --which surrogate_b2b,aucsort --sur-variants 0,15,16,17,18,19,0 \
    --reps 20 > gpurun_out/r02a_micro.jsonl 2> gpurun_out/r02a_micro.err
