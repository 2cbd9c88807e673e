#!/bin/bash
# round 3 re-entry: the whole GPU suite at HEAD, smoke, the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh pytest_gpu 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
ok $rc || exit $rc
for r in 1 2; do for d in 1 2 3 4; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_d$d.so python -u scripts/ab_eval.py 20 d$d >> gpurun_out/ab_depth.jsonl 2>>gpurun_out/ab_depth.err || exit $?
done; done
scripts/gpu_step.sh bench 480 python -u bench.py; rc=$?
exit $rc
