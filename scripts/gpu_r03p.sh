#!/bin/bash
# round 3: query ablation -- windows loaded but nothing counted (the count's VALU share)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do for v in tuning ab4; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_ab4.jsonl 2>>gpurun_out/ab_ab4.err || exit $?
done; done
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "surrogate" > gpurun_out/sur_tests_p.log 2>&1 || exit $?
