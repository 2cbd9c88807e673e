#!/bin/bash
# MIOpen exhaustive solver tuning (torch.backends.cudnn.benchmark = True) for the ResNet-50 b256
# channels-last bf16 step, into a user perf/find db under gpurun_out/ so it comes back; then the
# default-find step time with and without that db. A heartbeat line every 30 s marks progress
# while one find call tunes; every step has its own time limit.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
DB=gpurun_out/miopen_tuned; mkdir -p $DB /tmp/miopen_base
run() {  # name secs env... -- args
  name=$1; secs=$2; shift 2
  ( while sleep 30; do echo "[hb $name] $(date +%T) $(ls -la $DB 2>/dev/null | wc -l) db files"; done ) & hb=$!
  timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; rc=$?
  kill $hb; wait $hb 2>/dev/null
  echo "== $name exit $rc"; grep RESULT gpurun_out/$name.log; tail -3 gpurun_out/$name.log
  return $rc
}
run base 300 env MIOPEN_USER_DB_PATH=/tmp/miopen_base python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20; rc=$?
ok $rc || exit $rc
run tune 840 env MIOPEN_USER_DB_PATH=$DB python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20 --benchmark 1; rc=$?
ok $rc || exit $rc
run reuse 300 env MIOPEN_USER_DB_PATH=$DB python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20; rc=$?
ls -la $DB
exit $rc
