#!/bin/bash
# round-2 evidence: sharded-compaction smoke (2 gloo ranks through bench.py), kernel trace of the
# bench, PMC traffic (update, surrogate, compaction, query), and an interleaved surrogate A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02_prof gpurun_out/pmc_r02
timeout -k 10 600 python -u -m pytest -x -q --timeout 550 --timeout-method thread tests/test_bench_gpu.py \
    tests/test_kernels_gpu.py -k "bench or auc" > gpurun_out/r02_prof/tests.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof -o bench -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r02_prof/bench.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_r02 -o pmc_$c -- \
      python3 scripts/micro_kernels.py --which update,surrogate --variants 0 --reps 5 \
      > gpurun_out/pmc_r02/log_$c.txt 2>&1 || exit 1
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_r02 -o pmcq_$c -- \
      python3 scripts/probe_query.py 27 0.001 3 > gpurun_out/pmc_r02/logq_$c.txt 2>&1 || exit 1
done
for r in 1 2 3 4; do
  timeout -k 10 120 python3 scripts/micro_kernels.py --which surrogate_b2b --sur-variants 0,20,22,15 --reps 100 \
      >> gpurun_out/r02_prof/sur_ab.jsonl 2>/dev/null || exit 1
done
