#!/bin/bash
# rehearsal of the driver's N=8 path: 8 ranks over gloo sharing the one GPU (timings meaningless),
# and the 8-rank CoDA trajectory test on the device
set -o pipefail
mkdir -p gpurun_out/r02o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 380 --timeout-method thread \
    tests/test_coda_gpu.py -k "gloo_on_device" > gpurun_out/r02o/tests.log 2>&1 || exit 1
timeout -k 10 1000 python3 bench.py --gpus 8 --backend gloo --batch 32 --steps 4 --warmup 2 --sweep-I 1,8 \
    --sweep-steps 8 --r18-steps 4 --auc2-log2n 25 --cpu-sklearn-full 0 --sur-reps 10 --cpu-steps 8 \
    > gpurun_out/r02o/bench_n8_gloo.json 2> gpurun_out/r02o/bench_n8_gloo.err || exit 1
