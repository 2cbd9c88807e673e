#!/bin/bash
# HIP graph replay of the CoDA step: parity (vs eager and the reference), then the configs[0]
# GPU leg (ResNet-18 b32) with and without the graph
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02g2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_coda_gpu.py \
    > $O/tests.log 2>&1 || exit 1
for g in 1 0; do
  timeout -k 10 600 python3 bench.py --steps 5 --warmup 3 --sweep-I "" --no-auc --no-surrogate --no-cpu-baseline \
      --r18-steps 32 --r18-graph $g > $O/bench_r18_graph$g.json 2> $O/bench_r18_graph$g.err || exit 1
done
