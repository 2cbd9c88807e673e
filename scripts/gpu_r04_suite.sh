#!/bin/bash
# round 4: the whole GPU suite at HEAD (after the tuning-build-only staged-compaction variant)
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
D=gpurun_out/r04s2
mkdir -p $D
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1
rc=$?
echo "suite rc=$rc"
tail -3 $D/pytest_gpu.log
exit $rc
