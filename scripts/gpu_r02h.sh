#!/bin/bash
# full GPU suite (new: configs[0]/[1]/[4] real sizes, bench self-launch, INTEGRATION stub), then
# the pipelined query stream and surrogate reduce-rows timings
set -o pipefail
mkdir -p gpurun_out/r02h
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu \
    > gpurun_out/r02h/tests.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 > gpurun_out/r02h/micro.jsonl 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02h/trace -o run -- python3 scripts/probe_query.py 27 0.001 5 \
    > gpurun_out/r02h/trace.log 2>&1 || exit 1
for v in default rr256 rr1024; do
  lib=distributedauc_amd/libdauc.so; [ $v != default ] && lib=tuning/libdauc_$v.so
  DAUC_LIB=$lib timeout -k 10 120 python -u scripts/micro_kernels.py --which surrogate_b2b --sur-variants 0,15,0 --reps 30 \
      > gpurun_out/r02h/sur_$v.jsonl 2>&1 || exit 1
done
