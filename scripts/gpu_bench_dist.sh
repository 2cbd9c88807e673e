#!/bin/bash
# N=1 bench (all legs), then an N=2 rehearsal of the distributed bench path (gloo, both ranks on cuda:0)
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh bench 500 python -u bench.py ${BENCH_ARGS:-}; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh bench_n2_gloo 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 4 --warmup 2 --backend gloo \
    --auc2-log2n 0 --no-surrogate; rc=$?
exit $rc
