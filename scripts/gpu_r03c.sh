#!/bin/bash
# round 3: query-kernel A/B (phased LDS lookups, ping-pong pipeline), the tail-kernel stamps,
# the GPU suite on the new product / tuning split, the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
for v in p1u1 p0u2ph p0u4ph; do
  scripts/gpu_step.sh sort_$v 200 env DAUC_LIB=tuning/libdauc_$v.so python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "sorted or extreme or auc_counts_large or eval_counts or direct"; rc=$?
  ok $rc || exit $rc
done
for r in 1 2; do for v in p0u2 p1u1 p0u2ph p0u4ph; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_eval2.jsonl 2>>gpurun_out/ab_eval2.err || exit $?
done; done
cat gpurun_out/ab_eval2.jsonl
scripts/gpu_step.sh stamps 120 python -u scripts/probe_tail_stamps.py 20; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh pytest_gpu 480 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench 420 python -u bench.py --no-train --r18-steps 0; rc=$?
exit $rc
