#!/bin/bash
# round 6: the slotted two-step chain's geometry knobs (tuning build): the query grid's queries per
# thread and the compaction's fill stores per thread, G = 8 at both sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06knobs
mkdir -p $O
for rep in 1 2; do
for qpt in 4 8 16; do
  for fpt in 4 16; do
    DAUC_QUERY_QPT=$qpt DAUC_FILL_PER_THREAD=$fpt timeout -k 10 120 python -u scripts/probe_two_step.py 30 --trace --tuning \
        >> $O/knobs.jsonl 2>> $O/knobs.err || exit $?
  done
done
done
echo done
