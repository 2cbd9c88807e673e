#!/bin/bash
# the in-training AUC direction, fused/unfused, bf16/fp32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04diag
timeout -k 10 300 python -u scripts/diag_auc_direction.py --out gpurun_out/r04diag/default.json > gpurun_out/r04diag/default.log 2>&1 &&
timeout -k 10 300 python -u scripts/diag_auc_direction.py --fused-bn 0 --gemm 0 --out gpurun_out/r04diag/unfused.json > gpurun_out/r04diag/unfused.log 2>&1 &&
timeout -k 10 400 python -u scripts/diag_auc_direction.py --fused-bn 0 --gemm 0 --amp 0 --out gpurun_out/r04diag/fp32.json > gpurun_out/r04diag/fp32.log 2>&1
