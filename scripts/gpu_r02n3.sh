#!/bin/bash
# why is the graph-replayed configs[0] leg slow at 2 gloo ranks on one GPU: graph vs eager
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02n3
mkdir -p $O
for g in 1 0; do
  timeout -k 10 600 python3 bench.py --gpus 2 --backend gloo --batch 32 --steps 2 --warmup 1 --sweep-I "" \
      --r18-steps 8 --r18-graph $g --no-auc --no-surrogate --no-cpu-baseline > $O/bench_n2_g$g.json 2> $O/bench_n2_g$g.err || exit 1
done
