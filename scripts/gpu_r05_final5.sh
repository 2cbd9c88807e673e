#!/bin/bash
# round-5 evidence at HEAD (fifth pass: + stem XCD-aware tasks, wgrad XCD-aware (tile, split) placement): the whole GPU suite, smoke, the default bench line, the kernel trace of
# the bench, PMC traffic (update, loss, evaluation query). Every step under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
O=gpurun_out/r05final5
mkdir -p $O gpurun_out/pmc_r05e
DAUC_BENCH_RECORD_DIR=$O scripts/gpu_step.sh r05final5/pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh r05final5/smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 600 $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_trace.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_r05e -o pmc_$c -- \
      python3 scripts/micro_kernels.py --which update,surrogate --variants 0 --reps 5 \
      > gpurun_out/pmc_r05e/log_$c.txt 2>&1 || exit $?
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_r05e -o pmcq_$c -- \
      python3 scripts/probe_query.py 27 0.001 3 > gpurun_out/pmc_r05e/logq_$c.txt 2>&1 || exit $?
done
echo done
