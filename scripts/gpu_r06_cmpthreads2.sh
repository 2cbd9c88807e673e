#!/bin/bash
# round 6: 512 (the product's from 2^23 labels) against 1024 threads per compaction tile, three
# interleaved rounds (tuning build, DAUC_CMP_THREADS; scripts/probe_two_step.py --tuning, G = 2, 4, 8;
# every line's parts checked against the one-call evaluation).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06cmpthreads2
mkdir -p $O
for rep in 1 2 3; do
for t in 512 1024; do
  DAUC_CMP_THREADS=$t timeout -k 10 200 python -u scripts/probe_two_step.py 40 --tuning >> $O/probe.jsonl 2>> $O/probe.err || exit $?
done
done
echo done
