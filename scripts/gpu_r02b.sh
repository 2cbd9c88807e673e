#!/bin/bash
# round 2: compact-tree query kernel: parity (default build), then the tuning sweep of the
# query geometry (lockstep keys x max splitters x blocks per CU), one process per library
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "compact or nonfinite or extreme or sorted_counts or auc or radix" > gpurun_out/r02b_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 > gpurun_out/r02b_micro_default.jsonl 2>&1 || exit 1
for v in q1_s40000 q2_s40000 q1_s32767 q4_s32767 q1_s16383_b2 q2_s16383_b2; do
  DAUC_LIB=tuning/libdauc_$v.so timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 \
     > gpurun_out/r02b_micro_$v.jsonl 2>&1 || exit 1
done
