#!/bin/bash
# one-launch loss at stream occupancy (64 VGPRs): parity, then b2b timings vs the stream alone
set -o pipefail
mkdir -p gpurun_out/r02l
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_kernels_gpu.py \
    -k "surrogate" > gpurun_out/r02l/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 scripts/micro_kernels.py --which surrogate_b2b --sur-variants 0,15,25,21,22,23 --reps 100 \
      >> gpurun_out/r02l/sur_ab.jsonl 2>/dev/null || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02l/trace -o run -- \
    python3 scripts/micro_kernels.py --which surrogate_b2b --sur-variants 0,15 --reps 100 > gpurun_out/r02l/trace.log 2>&1 || exit 1
