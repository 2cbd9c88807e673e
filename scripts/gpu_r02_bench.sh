#!/bin/bash
# bench.py as the driver runs it (N=1 default), then a 2-rank self-launched gloo rehearsal with
# training (both ranks share cuda:0), short
set -o pipefail
mkdir -p gpurun_out/r02_bench
export TMPDIR=/tmp
( time timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ) > gpurun_out/r02_bench/n1.json 2> gpurun_out/r02_bench/n1.err || exit 1
timeout -k 10 600 python3 bench.py --gpus 2 --backend gloo --steps 8 --warmup 3 --sweep-steps 32 --r18-steps 8 \
    --auc-reps 1 --sur-reps 5 --no-cpu-baseline > gpurun_out/r02_bench/n2_gloo.json 2> gpurun_out/r02_bench/n2_gloo.err
