#!/bin/bash
# surrogate row-reduce A/B (0 = polling hand-off, 1 = last-arriver ticket): parity at 1, then the
# bench's surrogate leg alternating 0 / 1 / 0 / 1
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
DAUC_SURROGATE_REDUCE=1 scripts/gpu_step.sh pytest_sur1 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "surrogate or class_sums" --timeout 120 --timeout-method thread; rc=$?
ok $rc || exit $rc
for v in 0 1 0 1; do
  DAUC_SURROGATE_REDUCE=$v timeout -k 10 200 python -u bench.py --no-train --no-auc --no-cpu-baseline --sur-reps 50 > gpurun_out/sur_$v.log 2>&1
  rc=$?; echo "== reduce $v exit $rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/sur_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read())['surrogate_kernel']; print('reduce', $v, round(d['avg_launch_us'],2), round(d['per_call_events_us'],2), round(d['roofline']['frac'],4))"
done
