#!/bin/bash
# surrogate leg alone in a fresh process (memory-context check), then the query kernel's VALU PMC
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02x
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-train --no-auc --r18-steps 0 --no-cpu-baseline \
      >> gpurun_out/r02x/bench_sur_only.jsonl 2>> gpurun_out/r02x/bench_sur_only.err || exit 1
done
bash scripts/gpu_pmc_query_valu.sh || exit 1
