#!/bin/bash
# Surrogate row-reduce change: surrogate parity tests, the bench's surrogate leg, rocprof of it.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_sur 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "surrogate or class_sums" --timeout 120 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench_sur 300 python -u bench.py --no-train --no-auc --no-cpu-baseline --sur-reps 40; rc=$?
ok $rc || exit $rc
mkdir -p gpurun_out/prof_sur
scripts/gpu_step.sh rocprof_sur 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sur -o sur -- python -u bench.py --no-train --no-auc --no-cpu-baseline --sur-reps 40
