#!/bin/bash
# BN partial-pass workgroup size A/B (256 / 512 / 1024): parity tests at 1024, then kernel times
# from rocprofv3 with the 1x1 engines pinned
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp DAUC_CONV1X1=gemm
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
DAUC_BN_PART_THREADS=1024 scripts/gpu_step.sh pytest_bn1024 300 python -u -m pytest tests/test_fused_bn_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread; rc=$?
ok $rc || exit $rc
mkdir -p gpurun_out/abth
for v in 256 512 1024; do
  DAUC_BN_PART_THREADS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abth -o th$v -- \
      python -u bench.py --steps 10 --warmup 3 --no-auc --no-surrogate --no-cpu-baseline > gpurun_out/abth/log$v.txt 2>&1
  rc=$?; echo "== th$v exit $rc"
  [ $rc -eq 0 ] || exit $rc
done
