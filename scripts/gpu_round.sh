#!/bin/bash
# Standard GPU check: parity tests, smoke, short bench. Stops at the first
# step that ends in anything but pass/ordinary failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_gpu 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench 400 python -u bench.py ${BENCH_ARGS:-}; rc=$?
exit $rc
