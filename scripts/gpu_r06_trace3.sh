#!/bin/bash
# round 6 (end): kernel trace of one rank's two-step chain at G = 8 with the shipped kernels (grouped reduction, hoisted prologue loads, zeroing launch, 512-thread compaction tiles), both sizes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06trace3
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o two_step -- \
    python3 scripts/probe_two_step.py 20 --trace > $O/probe_trace.jsonl 2> $O/probe_trace.err; rc=$?
echo "rc=$rc"; cat $O/probe_trace.jsonl
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_by_grid.py "$f" $O/kernels_by_grid.json
exit $rc
