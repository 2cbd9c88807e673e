#!/bin/bash
# round 5: stride-2 wgrad layouts at the three ResNet-50 b256 stride-2 shapes: gather, shared rows
# 64 / 128 and the automatic choice (micro-benchmark), after the wgrad tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05z}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_wgrad_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest_wgrad.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; tail -1 $O/pytest_wgrad.log
[ $rc -eq 0 ] || exit $rc
for f in 1 4 5; do
    timeout -k 10 120 python3 scripts/probe_wgrad.py 20 $f >> $O/probe.jsonl 2>> $O/probe.err || exit $?
done
timeout -k 10 120 python3 scripts/probe_wgrad.py 20 >> $O/probe.jsonl 2>> $O/probe.err || exit $?
python3 -c "
import json
for l in open('$O/probe.jsonl'):
    d = json.loads(l); print(d['form'], d['C'], d['H'], d['stride'], round(d['us_per_call'], 1))"
