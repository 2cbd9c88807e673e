#!/bin/bash
# round 4: the query pass's fixed cost against the table size (the LDS index it loads)
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04k
mkdir -p $D
for p in 0.0001 0.00001; do
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof_$p -o run -- python3 $GRAFT_REPO_ROOT/scripts/probe_query_intercept.py 10 $p > $GRAFT_REPO_ROOT/$D/trace_$p.log 2>&1 || exit 1
done
