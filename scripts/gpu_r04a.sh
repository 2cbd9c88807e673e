#!/bin/bash
# round 4: the learning-direction test, the full 2-rank bench rehearsal, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04a
export DAUC_BENCH_RECORD_DIR=gpurun_out/r04a
timeout -k 10 600 python -u -m pytest tests/test_learning_gpu.py tests/test_bench_gpu.py -m gpu -x -v --timeout 900 --timeout-method thread > gpurun_out/r04a/new_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04a/pytest_gpu.log 2>&1
