#!/bin/bash
# round-6 closing check at HEAD (after the one-call count pass's single scan): the whole GPU suite and
# smoke, each under its own time limit; a failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
O=gpurun_out/r06final5
mkdir -p $O
DAUC_BENCH_RECORD_DIR=$O scripts/gpu_step.sh r06final5/pytest_gpu 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh r06final5/smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
exit $rc
