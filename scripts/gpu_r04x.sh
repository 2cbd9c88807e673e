#!/bin/bash
# round 4: the range-slot query path (tests, A/B against the count-index path, kernel traces),
# then the gather-thinning ablations (wrong counts by design), then the full GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04x
mkdir -p $D
cd $R
timeout -k 10 400 python -u -m pytest tests/test_auc_slots_gpu.py -x -v --timeout 300 --timeout-method thread > $D/pytest_slots.log 2>&1
rc=$?
echo "slots tests rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_eval_paths.py 20 3 > $D/ab_eval_paths.jsonl 2> $D/ab_eval_paths.err || exit 1
cd /tmp
DAUC_QUERY_PATH=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/p2 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/p2.log 2>&1 || exit 1
DAUC_QUERY_PATH=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/p2_24 -o run -- python3 $R/scripts/prof_eval.py 24 0.01 5 > $D/p2_24.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
for t in 1 3; do
  DAUC_LIB=$R/tuning/libdauc_t$t.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t$t -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t$t.log 2>&1 || exit 1
done
cd $R && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
