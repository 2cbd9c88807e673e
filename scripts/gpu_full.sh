#!/bin/bash
# parity tests -> kernel sweeps -> bench -> rocprofv3 kernel trace of the bench
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
R=${ROUND:-r01}
scripts/gpu_step.sh pytest_gpu 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread; rc=$?
ok $rc || exit $rc
if [ -z "$SKIP_MICRO" ]; then
scripts/gpu_step.sh micro_s4 200 python -u scripts/micro_kernels.py --which surrogate,update; rc=$?; ok $rc || exit $rc
for v in s2 s1; do
  [ -f tuning/libdauc_$v.so ] || continue
  DAUC_LIB=tuning/libdauc_$v.so scripts/gpu_step.sh micro_$v 200 python -u scripts/micro_kernels.py --which surrogate; rc=$?; ok $rc || exit $rc
done
fi
scripts/gpu_step.sh bench 500 python -u bench.py ${BENCH_ARGS:-}; rc=$?
ok $rc || exit $rc
mkdir -p gpurun_out/prof_$R
scripts/gpu_step.sh rocprof_bench 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o bench -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline; rc=$?
exit $rc
