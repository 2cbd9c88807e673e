#!/bin/bash
# backbone fast paths at the bench shape vs fp32 torch; bench stdout = the JSON record only
set -o pipefail
mkdir -p gpurun_out/r02n
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 880 --timeout-method thread \
    tests/test_conv1x1_gpu.py::test_resnet_fast_paths_at_bench_shape tests/test_bench_gpu.py \
    > gpurun_out/r02n/tests.log 2>&1 || exit 1
