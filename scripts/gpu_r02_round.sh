#!/bin/bash
# round-2 evidence pass: GPU parity suite, smoke, the default bench line, its kernel trace, and the
# PMC traffic of the roofline kernels (update, the one-launch loss, the AUC passes)
set -o pipefail
export TMPDIR=/tmp
R=${ROUND_TAG:-r02}
mkdir -p gpurun_out/$R gpurun_out/pmc_$R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests -m gpu \
    > gpurun_out/$R/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > gpurun_out/$R/bench_line.json 2> gpurun_out/$R/bench.err || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$R/prof -o bench -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$R/prof_bench.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$R -o pmc_$c -- \
      python3 scripts/micro_kernels.py --which update,surrogate --variants 0 --reps 5 \
      > gpurun_out/pmc_$R/log_$c.txt 2>&1 || exit 1
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$R -o pmcq_$c -- \
      python3 scripts/probe_query.py 27 0.001 3 > gpurun_out/pmc_$R/logq_$c.txt 2>&1 || exit 1
done
