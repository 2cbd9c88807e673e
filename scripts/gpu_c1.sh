#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_c1 300 python -u -m pytest tests/test_conv1x1_gpu.py -x -q --timeout 200 --timeout-method thread; rc=$?
ok $rc || exit $rc
[ $rc -eq 0 ] || exit 1
scripts/gpu_step.sh probe_f 200 python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --steps 10; rc=$?; ok $rc || exit $rc
scripts/gpu_step.sh probe_fg 200 python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 10; rc=$?; ok $rc || exit $rc
mkdir -p gpurun_out/prof_c1
scripts/gpu_step.sh rocprof_c1 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o probe -- python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 3; rc=$?
exit $rc
