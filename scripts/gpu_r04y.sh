#!/bin/bash
# round 4: LDS-lookup ablations of the count-index query (wrong counts by design), the range-slot
# tests, the two-step per-rank probe, then the full GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04y
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
DAUC_LIB=$R/tuning/libdauc_lin.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/lin -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/lin.log 2>&1 || exit 1
for a in 1 2 3; do
  DAUC_LIB=$R/tuning/libdauc_a$a.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/a$a -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/a$a.log 2>&1 || exit 1
done
cd $R
timeout -k 10 300 python -u scripts/probe_eval_part.py 20 > $D/eval_part_probe.jsonl 2> $D/eval_part_probe.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_auc_slots_gpu.py -v --timeout 300 --timeout-method thread > $D/pytest_slots.log 2>&1
rc=$?
echo "slots tests rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
echo "gpu suite rc=$?"
