#!/bin/bash
# round 3: box-to-box spread of the roofline kernels -- the loss call (product and its stream alone,
# variant 22), the update kernel and the 1 GiB D2D copy, HIP events, on whichever box this call gets
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/box
timeout -k 10 240 python -u scripts/micro_kernels.py --which surrogate,update,copy --variants 0 --sur-variants 0,22 --reps 50 >> gpurun_out/box/box_$(date +%s).jsonl 2>> gpurun_out/box/err.txt
