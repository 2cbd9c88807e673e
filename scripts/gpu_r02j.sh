#!/bin/bash
# branch-free bucket tail (query) + one-launch loss by default: parity, then timings
set -o pipefail
mkdir -p gpurun_out/r02j
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_kernels_gpu.py \
    tests/test_integration_gpu.py tests/test_coda_gpu.py > gpurun_out/r02j/tests.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02j/trace -o run -- python3 scripts/probe_query.py 27 0.001 5 \
    > gpurun_out/r02j/trace.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 > gpurun_out/r02j/micro.jsonl 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 scripts/micro_kernels.py --which surrogate_b2b --sur-variants 0,25,22,23,24,15 --reps 100 \
      >> gpurun_out/r02j/sur_ab.jsonl 2>/dev/null || exit 1
done
for v in spt8 spt4; do
  DAUC_LIB=tuning/libdauc_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
      tests/test_kernels_gpu.py -k "radix or sorted_counts or extreme" > gpurun_out/r02j/tests_$v.log 2>&1 || exit 1
  DAUC_LIB=tuning/libdauc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02j/trace_$v -o run -- \
      python3 scripts/probe_query.py 27 0.001 5 > gpurun_out/r02j/trace_$v.log 2>&1 || exit 1
done
