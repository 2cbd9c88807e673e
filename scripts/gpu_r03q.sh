#!/bin/bash
# round 3: the fingerprint form of the count index (DAUC_CI_FP = 2 / 3 keys per cell, one window per
# query: the two-window loop spills at 128 VGPRs) -- parity of the one-call evaluation, then the A/B
# against the product build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in fp2w fp3w; do
timeout -k 10 300 env DAUC_LIB=tuning/libdauc_$v.so python -u -m pytest tests/test_kernels_gpu.py tests/test_auc_cells_gpu.py -x -v --timeout 200 --timeout-method thread -k "sorted or extreme or eval or direct or count_index" > gpurun_out/${v}_tests.log 2>&1 || exit $?
done
for r in 1 2; do for v in tuning fp2w fp3w fp2wd; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_fpw.jsonl 2>>gpurun_out/ab_fpw.err || exit $?
done; done
