#!/bin/bash
# Second MIOpen tuning pass: MIOPEN_FIND_ENFORCE=SEARCH_DB_UPDATE re-tunes every tunable solver
# (also those the system perf db already covers), starting from the shipped db; then the
# default-find step time with the result. Heartbeat every 30 s; own time limits per step.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
DB=gpurun_out/miopen_tuned2; mkdir -p $DB; cp distributedauc_amd/miopen_db/* $DB/
run() {
  name=$1; secs=$2; shift 2
  ( while sleep 30; do echo "[hb $name] $(date +%T) $(wc -c < $DB/*.udb.txt) B udb"; done ) & hb=$!
  timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; rc=$?
  kill $hb; wait $hb 2>/dev/null
  echo "== $name exit $rc"; grep RESULT gpurun_out/$name.log; tail -2 gpurun_out/$name.log
  return $rc
}
run tune2 960 env MIOPEN_USER_DB_PATH=$DB MIOPEN_FIND_ENFORCE=SEARCH_DB_UPDATE python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20 --benchmark 1; rc=$?
ok $rc || exit $rc
run reuse2 300 env MIOPEN_USER_DB_PATH=$DB python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20; rc=$?
ok $rc || exit $rc
run reuse1 300 env MIOPEN_USER_DB_PATH=$PWD/distributedauc_amd/miopen_db python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20
