#!/bin/bash
# PyTorch TunableOp (hipBLASLt / rocBLAS solution search) for the ResNet-50 b256 backbone step's
# GEMMs, on top of the shipped MIOpen db: base, tuning run (results CSV under gpurun_out/), and a
# read-only reuse run of that CSV. Heartbeat every 30 s; each step has its own time limit.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
export MIOPEN_USER_DB_PATH=$PWD/distributedauc_amd/miopen_db
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
OUT=gpurun_out/tunableop; mkdir -p $OUT
run() {
  name=$1; secs=$2; shift 2
  ( while sleep 30; do echo "[hb $name] $(date +%T)"; done ) & hb=$!
  timeout -k 10 "$secs" "$@" > gpurun_out/$name.log 2>&1; rc=$?
  kill $hb; wait $hb 2>/dev/null
  echo "== $name exit $rc"; grep RESULT gpurun_out/$name.log; tail -2 gpurun_out/$name.log
  return $rc
}
run top_base 300 python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20; rc=$?
ok $rc || exit $rc
run top_tune 600 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/results%d.csv python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20; rc=$?
ok $rc || exit $rc
ls -la $OUT
run top_reuse 300 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/results%d.csv python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --gemm1x1 1 --steps 20
