#!/bin/bash
# round 6: the slotted query pass's end-of-kernel atomics (tuning build, DAUC_QUERY_ABL timing
# ablations; wrong counts by design, so only timed): 0 normal, 1 no query loop, 3 no atomics,
# 4 neither (the prologue only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06abl2
mkdir -p $O
for rep in 1 2; do
for abl in 0 1 3 4; do
  DAUC_QUERY_ABL=$abl timeout -k 10 120 python -u scripts/probe_query_abl.py 40 >> $O/abl.jsonl 2>> $O/abl.err || exit $?
done
done
echo done
