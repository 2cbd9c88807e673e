#!/bin/bash
# stability: the GPU suite twice in a row, smoke, and the N=4 gloo rehearsal of the bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02stab
mkdir -p $O
for r in 1 2; do
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests -m gpu \
      > $O/pytest_gpu_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python3 bench.py --gpus 4 --backend gloo --batch 32 --steps 4 --warmup 2 --sweep-I 1,8 \
    --sweep-steps 8 --r18-steps 8 --auc2-log2n 26 --cpu-sklearn-full 0 --sur-reps 10 --cpu-steps 8 \
    > $O/bench_n4.json 2> $O/bench_n4.err || exit 1
