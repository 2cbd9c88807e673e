#!/bin/bash
# round 4: the compaction's staged-score variant (tuning build) against the product form (A/B,
# counts compared)
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04g
mkdir -p $D
timeout -k 10 300 python -u scripts/ab_compact_stage.py 50 > $D/ab_compact_stage.jsonl 2> $D/ab_compact_stage.err || exit 1
