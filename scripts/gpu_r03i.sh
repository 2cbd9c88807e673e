#!/bin/bash
# round 3: eval determinism under cudnn.deterministic; query-kernel ablations (gathers / LDS lookups / U=2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
mkdir -p gpurun_out
scripts/gpu_step.sh det2 180 python -u scripts/probe_eval_determinism.py 48 det; rc=$?
ok $rc || exit $rc
scripts/gpu_step.sh det3 180 python -u scripts/probe_eval_determinism.py 48 algos; rc=$?
ok $rc || exit $rc
for r in 1 2; do for v in tuning ab1 ab2 ab3 u2; do
  timeout -k 10 120 env DAUC_LIB=tuning/libdauc_$v.so python -u scripts/ab_eval.py 20 $v >> gpurun_out/ab_abl.jsonl 2>>gpurun_out/ab_abl.err || exit $?
done; done
