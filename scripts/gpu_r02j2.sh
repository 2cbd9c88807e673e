#!/bin/bash
# end-to-end rehearsal of the driver's multi-rank bench at HEAD: 2 gloo ranks sharing cuda:0, every leg
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02j2
timeout -k 10 900 python3 bench.py --gpus 2 --backend gloo --steps 4 --warmup 2 \
    > gpurun_out/r02j2/bench_n2_gloo_full.json 2> gpurun_out/r02j2/bench_n2.err || exit 1
