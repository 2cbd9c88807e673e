#!/bin/bash
# the same configurations as the CPU oracle loop (scripts/cpu_oracle_direction.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04diag2
D=gpurun_out/r04diag2
timeout -k 10 300 python -u scripts/diag_auc_direction.py --arch resnet18 --image-size 32 --batch 64 --marks 0,10,25,50,100,150 --eval-images 2048 --out $D/r18_32.json > $D/r18_32.log 2>&1 &&
timeout -k 10 300 python -u scripts/diag_auc_direction.py --arch resnet50 --image-size 64 --batch 64 --marks 0,5,10,25,50 --eval-images 2048 --out $D/r50_64.json > $D/r50_64.log 2>&1 &&
timeout -k 10 300 python -u scripts/diag_auc_direction.py --lr 0.01 --marks 0,10,25,50,100,150 --out $D/r50_224_lr001.json > $D/r50_224_lr001.log 2>&1 &&
timeout -k 10 300 python -u scripts/diag_auc_direction.py --lr 0.001 --marks 0,10,25,50,100,150 --out $D/r50_224_lr0001.json > $D/r50_224_lr0001.log 2>&1
