#!/bin/bash
# (1) re-measure the 1x1-conv engine plan with the in-place accumulate; (2) train-only A/B: the new
# plan vs per-run timing (auto); (3) surrogate in-launch reduce variants: parity + timings
set -o pipefail
mkdir -p gpurun_out/r02i
export TMPDIR=/tmp
DAUC_CONV1X1_PLANS="" timeout -k 10 300 python -u scripts/gen_conv1x1_plans.py gpurun_out/r02i/conv1x1_plans.json \
    > gpurun_out/r02i/plans.log 2>&1 || exit 1
for mode in plan auto plan auto; do
  if [ $mode = plan ]; then P=gpurun_out/r02i/conv1x1_plans.json; else P=""; fi
  DAUC_CONV1X1_PLANS=$P timeout -k 10 300 python3 bench.py --no-auc --no-surrogate --no-cpu-baseline --sweep-I "" \
      --r18-steps 0 --steps 30 --warmup 5 >> gpurun_out/r02i/ab_$mode.jsonl 2>> gpurun_out/r02i/ab.err || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "chunked_variants or surrogate" > gpurun_out/r02i/sur_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_kernels.py --which surrogate_b2b --sur-variants 0,20,21,22,15,0,20 --reps 30 \
    > gpurun_out/r02i/sur.jsonl 2>&1
