#!/bin/bash
# round 5: stem staging with a wave-uniform fast path for whole-in-image chunks and the forward's
# staged chunks bounded by the pixels it reads. Stem tests, micro-benchmark of both builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ah}
PREV=${PREV:-tuning/ab/libdauc_st.so}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_stem_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_stem.log 2>&1
rc=$?; echo "stem tests rc=$rc"; tail -1 $O/pytest_stem.log
[ $rc -eq 0 ] || exit $rc
DAUC_LIB=$PREV timeout -k 10 120 python3 scripts/probe_stem.py 20 > $O/probe_prev.jsonl 2> $O/probe.err || exit $?
timeout -k 10 120 python3 scripts/probe_stem.py 20 > $O/probe_new.jsonl 2>> $O/probe.err || exit $?
head -2 $O/probe_prev.jsonl; head -2 $O/probe_new.jsonl
