#!/bin/bash
# round 4: stream-depth and stream-only variants of the count-index query (s*: wrong counts by
# design), the per-rank device-time probe, and the two re-expected tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04z
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
for v in s1 s4 d2 d4 w1 w4 w8 wu; do
  DAUC_LIB=$R/tuning/libdauc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/$v -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/$v.log 2>&1 || exit 1
done
cd $R
timeout -k 10 300 python -u scripts/probe_eval_part.py 20 > $D/eval_part_probe.jsonl 2> $D/eval_part_probe.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_auc_slots_gpu.py "tests/test_kernels_gpu.py::test_auc_eval_two_step_parts" -v --timeout 300 --timeout-method thread > $D/pytest_fix.log 2>&1
echo "tests rc=$?"
