#!/bin/bash
# round 3: query count variants (late windows, med3 counts): parity + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
for v in lw m3 lwm3; do
  scripts/gpu_step.sh t_$v 300 env DAUC_LIB=tuning/libdauc_$v.so python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py -x -q --timeout 150 --timeout-method thread -k "sorted or extreme or auc_counts_large or eval or direct or count_index"; rc=$?
  ok $rc || exit $rc
done
for r in 1 2; do for v in tuning lw m3 lwm3; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_lw.jsonl 2>>gpurun_out/ab_lw.err || exit $?
done; done
