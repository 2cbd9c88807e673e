#!/bin/bash
# the bench line at HEAD (AUC wall and event loops separated) and a 2-rank gloo rehearsal of the
# sharded sort-method legs (2^24 and 2^27: both shard now; both ranks on cuda:0)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02g
timeout -k 10 600 python3 bench.py > gpurun_out/r02g/bench_line.json 2> gpurun_out/r02g/bench.err || exit 1
timeout -k 10 400 python3 bench.py --gpus 2 --backend gloo --no-train --no-surrogate --no-cpu-baseline --auc-reps 2 \
    > gpurun_out/r02g/bench_n2_gloo_auc.json 2> gpurun_out/r02g/bench_n2.err || exit 1
