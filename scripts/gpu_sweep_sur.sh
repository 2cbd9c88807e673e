#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
for f in tuning/libdauc_s*.so; do
  DAUC_LIB=$f timeout -k 10 60 python -u scripts/micro_kernels.py --which surrogate --reps 20 >> gpurun_out/sweep_sur.log 2>&1
  rc=$?; echo "$f exit $rc"; [ $rc -eq 0 ] || exit $rc
done
