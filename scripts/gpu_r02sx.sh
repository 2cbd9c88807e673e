#!/bin/bash
# loss kernel: reducers as extra workgroups (variants 26-28) vs the last streaming workgroups
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02sy
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_kernels_gpu.py \
    -k "surrogate_chunked" > $O/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 scripts/micro_kernels.py --which surrogate_b2b --sur-variants 22,15,29,22,15,29 --reps 100 \
      >> $O/sur_ab.jsonl 2>/dev/null || exit 1
done
