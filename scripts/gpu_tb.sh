#!/bin/bash
# selected parity tests (TESTS, default: the whole GPU suite), then a short training-step bench
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_tb 400 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench_train 400 python -u bench.py --steps 20 --warmup 5 --no-auc --no-surrogate --no-cpu-baseline; rc=$?
exit $rc
