#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh bench 600 python -u bench.py; rc=$?
ok $rc || exit $rc
# multi-rank rehearsal of the driver's torchrun launch: 2 ranks share the one GPU over gloo
scripts/gpu_step.sh bench_2rank 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 \
    --batch 64 --auc-log2n 20 --auc-reps 1
