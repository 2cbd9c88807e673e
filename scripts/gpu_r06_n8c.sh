#!/bin/bash
# the driver's exact N>1 bench at full BASELINE sizes, 8 gloo ranks sharing cuda:0
# (R-50 b256 224^2 I=16, period sweep, sharded configs[3]/[4], CPU baselines on rank 0), after the
# INTEGRATION stub's GPU tests. Rerun at the end of round 6 with the two-step changes.
set -o pipefail
out=gpurun_out/r06n8c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_integration_gpu.py > $out/pytest_integration.log 2>&1 || {
    echo "pytest exit $?"; tail -30 $out/pytest_integration.log; exit 1; }
tail -3 $out/pytest_integration.log
timeout -k 10 900 python -u bench.py --gpus 8 --backend gloo --cpu-baseline-any-n > $out/bench_n8.json 2> $out/bench_n8.err
rc=$?
echo "bench exit $rc" | tee -a $out/bench_n8.err
tail -5 $out/bench_n8.err
exit $rc
