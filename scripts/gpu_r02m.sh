#!/bin/bash
# order effect in the loss micro-benchmark: the same kernel under two variant numbers
set -o pipefail
mkdir -p gpurun_out/r02m
for r in 1 2; do
  timeout -k 10 120 python3 scripts/micro_kernels.py --which surrogate_b2b --sur-variants 22,0,22,0,15,0,22 --reps 100 \
      >> gpurun_out/r02m/sur_order.jsonl 2>/dev/null || exit 1
done
