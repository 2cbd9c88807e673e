#!/bin/bash
# round 6: does the compaction's reservation (one returning atomic per tile on the slot's counter)
# bound step 1? Tuning build, DAUC_CMP_ABL = 1 (every tile writes from position 0, no atomic; wrong
# output by design, timed only) against 0, both sizes at G = 8 (scripts/probe_query_abl.py: ms_compact).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06cmpabl
mkdir -p $O
for rep in 1 2; do
for abl in 0 1; do
  DAUC_CMP_ABL=$abl timeout -k 10 120 python -u scripts/probe_query_abl.py 40 | sed "s/^{/{\"cmp_abl\": $abl, /" >> $O/abl.jsonl 2>> $O/abl.err || exit $?
done
done
echo done
