#!/bin/bash
# round 3: eval-forward determinism probe; COUNT3 query A/B + its parity tests; loss tail variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh det 180 python -u scripts/probe_eval_determinism.py 48; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh c3_tests 300 env DAUC_LIB=tuning/libdauc_c3.so python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py -x -q --timeout 150 --timeout-method thread -k "sorted or extreme or auc_counts_large or eval or direct or count_index"; rc=$?
ok $rc || exit $rc
for r in 1 2; do for v in c3 tuning; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_c3.jsonl 2>>gpurun_out/ab_c3.err || exit $?
done; done
scripts/gpu_step.sh ab_sur 240 python -u scripts/ab_surrogate.py 3 100 0,4,11,16,17,18,19,20; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh stamps21 120 python -u scripts/probe_tail_stamps.py 15 21; rc=$?
exit $rc
