#!/bin/bash
# 2-rank rehearsal of the full bench (gloo, shared GPU, small batch) with the graph-replayed
# configs[0] leg, plus the graph parity test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02n2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_coda_gpu.py -k graph \
    > $O/tests.log 2>&1 || exit 1
timeout -k 10 900 python3 bench.py --gpus 2 --backend gloo --batch 32 --steps 4 --warmup 2 --sweep-I 1,8 \
    --sweep-steps 8 --r18-steps 8 --auc2-log2n 25 --cpu-sklearn-full 0 --sur-reps 10 --cpu-steps 8 \
    > $O/bench_n2.json 2> $O/bench_n2.err || exit 1
