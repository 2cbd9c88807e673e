#!/bin/bash
# Surrogate chunk-kernel experiments: each tuning/libdauc_*.so is one compile-time variant.
cd "${GRAFT_REPO_ROOT:-.}"
for r in 1 2; do
for f in distributedauc_amd/libdauc.so tuning/libdauc_*.so; do
  echo "== $f" >> gpurun_out/sur_exp.log
  DAUC_LIB=$f timeout -k 10 60 python -u scripts/micro_kernels.py --which surrogate --reps 100 --sur-variants ${SUR_VARIANTS:-0,2} >> gpurun_out/sur_exp.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$f exit $rc"; exit $rc; }
done
done
