#!/bin/bash
# round 4: query-kernel structure experiments (g*: wrong counts by design): 512-thread workgroups
# with 1 / 4 / 8 stream groups, no gathers, no gathers and no block-word reads
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04w
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
for v in w1 w4 w8 g8 g10; do
  DAUC_LIB=$R/tuning/libdauc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/$v -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/$v.log 2>&1 || exit 1
done
