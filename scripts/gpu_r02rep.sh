#!/bin/bash
# AUC at 2 ranks (gloo, one GPU): 2^24 replicated, 2^27 sharded; the self-launch test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02rep
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 350 --timeout-method thread tests/test_bench_gpu.py \
    > $O/tests.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --gpus 2 --backend gloo --no-train --no-surrogate --no-cpu-baseline \
    > $O/bench_auc_n2.json 2> $O/bench_auc_n2.err || exit 1
