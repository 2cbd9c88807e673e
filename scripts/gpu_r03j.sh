#!/bin/bash
# round 3: 4-stage query pipeline A/B + parity; split-scoring test with deterministic eval; loss tests on the new tail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh p2_tests 300 env DAUC_LIB=tuning/libdauc_p2.so python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py -x -q --timeout 150 --timeout-method thread -k "sorted or extreme or auc_counts_large or eval or direct or count_index or surrogate"; rc=$?
ok $rc || exit $rc
for r in 1 2; do for v in tuning p2 p2d2 p2ab2; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_p2.jsonl 2>>gpurun_out/ab_p2.err || exit $?
done; done
scripts/gpu_step.sh split 420 python -u -m pytest tests/test_main_gpu.py -x -v --timeout 400 --timeout-method thread; rc=$?
exit $rc
