#!/bin/bash
# round 4: the narrow compaction tiles' size (A/B) and the slot tests
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04j
mkdir -p $D
timeout -k 10 300 python -u scripts/ab_compact_slots.py 50 > $D/ab_compact_slots.jsonl 2> $D/ab_compact_slots.err || exit 1
