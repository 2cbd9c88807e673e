#!/bin/bash
# round 3: non-temporal window gathers A/B + parity
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh t_wnt 300 env DAUC_LIB=tuning/libdauc_wnt.so python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "sorted or extreme or eval or direct or count_index"; rc=$?
ok $rc || exit $rc
for r in 1 2 3; do for v in tuning wnt; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_wnt.jsonl 2>>gpurun_out/ab_wnt.err || exit $?
done; done
