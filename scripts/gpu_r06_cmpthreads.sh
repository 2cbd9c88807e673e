#!/bin/bash
# round 6: larger compaction workgroups below 2^25 labels (tuning build, DAUC_CMP_THREADS = 512 / 1024
# threads per tile of 8 label groups per thread, against the product's 256): fewer tiles, fewer
# reservations on the slot's one counter. scripts/probe_two_step.py --tuning, interleaved twice; the
# parts' counts are checked against the one-call evaluation in every line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06cmpthreads
mkdir -p $O
for rep in 1 2; do
for t in 256 512 1024; do
  if [ $t = 256 ]; then unset DAUC_CMP_THREADS; else export DAUC_CMP_THREADS=$t; fi
  timeout -k 10 200 python -u scripts/probe_two_step.py 40 --tuning >> $O/probe.jsonl 2>> $O/probe.err || exit $?
done
done
echo done
