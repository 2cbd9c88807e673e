#!/bin/bash
# round 3: second-window prefetch (W2) parity + A/B; split-scoring test; product loss tail tests + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh w2_tests 300 env DAUC_LIB=tuning/libdauc_w2.so python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py -x -q --timeout 150 --timeout-method thread -k "sorted or extreme or auc_counts_large or eval or direct or count_index"; rc=$?
ok $rc || exit $rc
for r in 1 2; do for v in tuning w2; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_w2.jsonl 2>>gpurun_out/ab_w2.err || exit $?
done; done
scripts/gpu_step.sh sur_tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "surrogate or class_sums or logits"; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh ab_sur 240 python -u scripts/ab_surrogate.py 3 100 0,3,20,22; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh split 420 python -u -m pytest tests/test_main_gpu.py -x -v --timeout 400 --timeout-method thread; rc=$?
exit $rc
