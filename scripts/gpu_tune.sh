#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh micro 300 python -u scripts/micro_kernels.py; rc=$?
ok $rc || exit $rc
scripts/probe_backbone.sh
