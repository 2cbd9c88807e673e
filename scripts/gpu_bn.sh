#!/bin/bash
# fused BN kernels: parity tests, then backbone step time fused vs unfused (row-block sweep), rocprof
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
scripts/gpu_step.sh pytest_bn 300 python -u -m pytest tests/test_fused_bn_gpu.py -x -q --timeout 120 --timeout-method thread; rc=$?
ok $rc || exit $rc
[ $rc -eq 0 ] || exit 1
[ -n "$NO_UNFUSED" ] || { scripts/gpu_step.sh probe_unfused 200 python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 0; rc=$?; ok $rc || exit $rc; }
for rb in ${ROWBLOCKS:-512}; do
  DAUC_BN_ROWBLOCKS=$rb scripts/gpu_step.sh probe_fused_$rb 200 python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --steps 10; rc=$?; ok $rc || exit $rc
done
mkdir -p gpurun_out/prof_bn
scripts/gpu_step.sh rocprof_probe 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bn -o probe -- python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --steps 3; rc=$?
exit $rc
