#!/bin/bash
# query_ci unroll (float4 slots per iteration): U = 2 (product), 3, 4 via tuning builds
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ci_u
timeout -k 10 120 python -u scripts/probe_eval_part.py 30 > gpurun_out/ci_u/u2.jsonl 2>&1 || exit 1
for u in 3 4; do
  DAUC_LIB=tuning/libdauc_u$u.so timeout -k 10 120 python -u scripts/probe_eval_part.py 30 > gpurun_out/ci_u/u$u.jsonl 2>&1 || exit 1
done
DAUC_LIB=tuning/libdauc_u3.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ci_u/t3 -o run -- \
    python3 scripts/probe_eval_part.py 3 > gpurun_out/ci_u/t3.log 2>&1 || exit 1
DAUC_LIB=tuning/libdauc_u4.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ci_u/t4 -o run -- \
    python3 scripts/probe_eval_part.py 3 > gpurun_out/ci_u/t4.log 2>&1 || exit 1
