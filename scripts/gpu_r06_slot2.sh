#!/bin/bash
# round 6: the slotted build in the one-call evaluation too -- the AUC GPU tests, smoke, the A/B
# probe of both index forms (two-step parts and the one-call evaluation), then the N=1 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06slot2
mkdir -p $O
scripts/gpu_step.sh r06slot2/pytest_auc 420 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_two_step_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py tests/test_main_gpu.py \
    tests/test_kernels_gpu.py -k "auc or eval or two_step or count or split or pair or sort or index or main"; rc=$?
[ $rc -eq 0 ] || exit $rc
scripts/gpu_step.sh r06slot2/smoke 150 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 30 --ab > $O/probe_ab.jsonl 2> $O/probe_ab.err; rc=$?
echo "probe rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc"; tail -c 400 $O/bench.json
exit $rc
