#!/bin/bash
# exact-AUC kernels: parity tests, the bench's AUC legs, and their kernel times from rocprofv3
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_auc 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench_auc 300 python -u bench.py --no-train --no-surrogate --no-cpu-baseline; rc=$?
ok $rc || exit $rc
mkdir -p gpurun_out/prof_auc
scripts/gpu_step.sh rocprof_auc 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_auc -o auc -- python -u bench.py --no-train --no-surrogate --no-cpu-baseline
