#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
run() { echo "--- $*"; timeout -k 10 200 "$@" 2>&1 | grep -E "RESULT|Error|error" ; rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc; }
export MIOPEN_LOG_LEVEL=1
run env MIOPEN_FIND_MODE=FAST python -u scripts/probe_backbone.py --layout cl --dtype bf16
run env MIOPEN_FIND_MODE=FAST python -u scripts/probe_backbone.py --layout nchw --dtype bf16
run python -u scripts/probe_backbone.py --layout cl --dtype bf16
run python -u scripts/probe_backbone.py --layout nchw --dtype bf16
run python -u scripts/probe_backbone.py --layout cl --dtype bf16 --benchmark 1
run python -u scripts/probe_backbone.py --layout nchw --dtype bf16 --benchmark 1
run python -u scripts/probe_backbone.py --layout nchw --dtype fp32
