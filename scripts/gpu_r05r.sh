#!/bin/bash
# round 5: stem kernels with the staging loads in flight across the MFMAs. Stem parity tests and
# the micro-benchmark against MIOpen.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05r}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_stem_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest_stem.log 2>&1
rc=$?; echo "stem tests rc=$rc"; tail -3 $O/pytest_stem.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/probe_stem.py 20 > $O/probe_stem.jsonl 2> $O/probe_stem.err || exit $?
cat $O/probe_stem.jsonl
