#!/bin/bash
# round 3: query ablations on top of the straddling-window fix; per-rank sharded evaluation cost
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/probe_eval_part.py 30 > gpurun_out/eval_part.jsonl 2> gpurun_out/eval_part.err || exit $?
for r in 1 2; do for v in tuning wab1 wab2 wab3; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_wab.jsonl 2>>gpurun_out/ab_wab.err || exit $?
done; done
timeout -k 10 480 python -u bench.py --no-cpu-baseline > gpurun_out/bench_m.log 2>&1 || exit $?
timeout -k 10 420 python -u -m pytest tests/test_main_gpu.py -x -q --timeout 400 --timeout-method thread > gpurun_out/main_m.log 2>&1 || exit $?
