#!/bin/bash
# 3-ary (ds_read_b64) vs 5-ary (ds_read_b128) search tree: parity of the 3-ary build, then timings
set -o pipefail
mkdir -p gpurun_out/r02f
export TMPDIR=/tmp
DAUC_LIB=tuning/libdauc_a3.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "nonfinite or extreme or sorted_counts or auc" > gpurun_out/r02f/tests_a3.log 2>&1 || exit 1
for v in default a3 a3_abl1; do
  lib=distributedauc_amd/libdauc.so; [ $v != default ] && lib=tuning/libdauc_$v.so
  DAUC_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02f/$v -o run -- \
      python3 scripts/probe_query.py 27 0.001 5 > gpurun_out/r02f/$v.log 2>&1 || exit 1
  DAUC_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02f/${v}_24 -o run -- \
      python3 scripts/probe_query.py 24 0.01 5 > gpurun_out/r02f/${v}_24.log 2>&1 || exit 1
done
