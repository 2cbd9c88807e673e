#!/bin/bash
# round 4: the query pass's fixed cost (query_part at G = 8 .. 1024 under a kernel trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04m
mkdir -p $D
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/probe_query_intercept.py 10 > $GRAFT_REPO_ROOT/$D/trace.log 2>&1 || exit 1
