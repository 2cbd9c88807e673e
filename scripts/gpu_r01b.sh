#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh micro_s4 200 python -u scripts/micro_kernels.py --which surrogate; rc=$?; ok $rc || exit $rc
for v in s2 s8; do
  DAUC_LIB=tuning/libdauc_$v.so scripts/gpu_step.sh micro_$v 200 python -u scripts/micro_kernels.py --which surrogate; rc=$?; ok $rc || exit $rc
done
scripts/gpu_pmc.sh
