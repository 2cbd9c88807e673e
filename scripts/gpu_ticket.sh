#!/bin/bash
# single-launch ticket surrogate: parity (all variants, shared workspace), then timing vs the two-launch form
cd "${GRAFT_REPO_ROOT:-.}"
scripts/gpu_step.sh pytest_ticket 300 python -u -m pytest tests/test_kernels_gpu.py -k "surrogate_chunked" -x -v --timeout 150 --timeout-method thread || exit $?
scripts/gpu_step.sh micro_ticket 300 python -u scripts/micro_kernels.py --which surrogate --sur-variants 0,8,9,10,11,12,13,14 --reps 30
