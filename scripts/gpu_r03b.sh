#!/bin/bash
# round 3: configs[2] 8-rank test; A/B of the pipelined count-index query; GPU suite; bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh sorttests_p1u1 300 env DAUC_LIB=tuning/libdauc_p1u1.so python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 250 --timeout-method thread -k "sorted or extreme or auc_counts_large or eval_counts or direct"; rc=$?
ok $rc || exit $rc
for r in 1 2; do for v in p0u2 p1u1 p1u2; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_eval.jsonl 2>>gpurun_out/ab_eval.err || exit $?
done; done
cat gpurun_out/ab_eval.jsonl
scripts/gpu_step.sh configs2 700 python -u -m pytest tests/test_configs2_gpu.py -x -v --timeout 680 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh pytest_gpu 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread --deselect tests/test_configs2_gpu.py::test_configs2_resnet50_8ranks_period_sweep; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench 420 python -u bench.py; rc=$?
exit $rc
