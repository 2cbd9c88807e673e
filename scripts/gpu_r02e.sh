#!/bin/bash
# query kernel ablations (timing only): normal / no bucket load / no tree walk
set -o pipefail
mkdir -p gpurun_out/r02e
export TMPDIR=/tmp
for v in default abl1 abl2; do
  lib=distributedauc_amd/libdauc.so; [ $v != default ] && lib=tuning/libdauc_$v.so
  DAUC_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02e/$v -o run -- \
      python3 scripts/probe_query.py 27 0.001 5 > gpurun_out/r02e/$v.log 2>&1 || exit 1
done
