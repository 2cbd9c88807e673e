#!/bin/bash
# round-6 evidence at HEAD after the two-step changes (grouped reduction, prologue hoist, zeroing launch, 512-thread compaction tiles, one-scan count pass):
# the whole GPU suite, smoke, the default N=1 bench line, then the per-rank two-step probe (product,
# G = 2, 4, 8). Every step under its own time limit; an abort / timeout ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
O=gpurun_out/r06final4
mkdir -p $O
DAUC_BENCH_RECORD_DIR=$O scripts/gpu_step.sh r06final4/pytest_gpu 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh r06final4/smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 600 $O/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 40 > $O/probe_two_step.jsonl 2> $O/probe_two_step.err; rc=$?
echo "probe rc=$rc"
exit $rc
