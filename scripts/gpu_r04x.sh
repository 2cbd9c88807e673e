#!/bin/bash
# temporary: count-kernel ablations (wrong counts by design) at 2^27, kernel trace per library
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04x
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
for t in 1 3; do
  DAUC_LIB=$R/tuning/libdauc_t$t.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t$t -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t$t.log 2>&1 || exit 1
done
for x in 0 1 2 3; do
  L=$R/tuning/libdauc_x$x.so
  DAUC_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/x$x -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/x$x.log 2>&1 || exit 1
done
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
