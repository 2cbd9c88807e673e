#!/bin/bash
# round 4: the compaction's tile size (A/B), the slot layout test and the two-step tests
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04n
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -k "two_step or slot_layout or eval" --timeout 200 --timeout-method thread > $D/pytest_slots.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_compact_wide.py 50 > $D/ab_compact_wide.jsonl 2> $D/ab_compact_wide.err || exit 1
