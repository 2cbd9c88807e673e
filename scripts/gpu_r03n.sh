#!/bin/bash
# round 3: wide compaction workgroups (512 / 1024 threads) parity + A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
for v in cw1024 cw512; do
  scripts/gpu_step.sh t_$v 300 env DAUC_LIB=tuning/libdauc_$v.so python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread -k "extreme or eval or compact"; rc=$?
  ok $rc || exit $rc
done
for r in 1 2; do for v in tuning cw1024 cw512; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_cw.jsonl 2>>gpurun_out/ab_cw.err || exit $?
done; done
export DAUC_LIB=tuning/libdauc_cw1024.so
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cwtrace -o cw -- python3 scripts/ab_eval.py 5 cw1024 > gpurun_out/cwtrace.log 2>&1 || exit $?
