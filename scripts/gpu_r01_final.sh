#!/bin/bash
# Round evidence: full GPU parity suite, smoke, bench, rocprofv3 kernel trace of the bench,
# PMC traffic passes. Stops at the first step that ends in anything but pass/ordinary failure.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
R=${ROUND:-r01}
scripts/gpu_step.sh pytest_gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh bench 500 python -u bench.py ${BENCH_ARGS:-}; rc=$?
ok $rc || exit $rc
mkdir -p gpurun_out/prof_$R
scripts/gpu_step.sh rocprof_bench 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o bench -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline; rc=$?
ok $rc || exit $rc
bash scripts/gpu_pmc.sh
