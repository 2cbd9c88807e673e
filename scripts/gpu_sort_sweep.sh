#!/bin/bash
# Sorted-count (query kernel) geometry sweep: each tuning/libdauc_q_*.so is one compile-time variant.
cd "${GRAFT_REPO_ROOT:-.}"
export DAUC_MICRO_SORT_ONLY=1
for f in distributedauc_amd/libdauc.so tuning/libdauc_q_*.so; do
  echo "== $f" >> gpurun_out/sort_sweep.log
  DAUC_LIB=$f timeout -k 10 60 python -u scripts/micro_kernels.py --which paircount --reps 30 >> gpurun_out/sort_sweep.log 2>&1 || { echo "$f failed"; exit 1; }
  DAUC_MICRO_POS_RATE=0.001 DAUC_LIB=$f timeout -k 10 60 python -u scripts/micro_kernels.py --which paircount --reps 30 --log2n 27 >> gpurun_out/sort_sweep.log 2>&1 || { echo "$f failed"; exit 1; }
done
