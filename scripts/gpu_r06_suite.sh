#!/bin/bash
# round-6 evidence: the whole GPU suite, smoke, the default N=1 bench line (every step under its own
# time limit; an abort / timeout ends the call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
O=gpurun_out/r06final
mkdir -p $O
DAUC_BENCH_RECORD_DIR=$O scripts/gpu_step.sh r06final/pytest_gpu 560 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh r06final/smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 600 $O/bench.json
exit $rc
