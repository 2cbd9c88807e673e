#!/bin/bash
# backbone step time (fused BN) under MIOpen solver restrictions; one fresh find-db per config
cd "${GRAFT_REPO_ROOT:-.}"
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
export DAUC_BN_ROWBLOCKS=${DAUC_BN_ROWBLOCKS:-256}
i=0
while read -r cfg; do
  i=$((i+1)); db=/tmp/miopen_db_$i; mkdir -p $db
  echo "== config $i: ${cfg:-default}"
  env MIOPEN_USER_DB_PATH=$db $cfg timeout -k 10 240 python -u scripts/probe_backbone.py --layout cl --dtype bf16 --fused 1 --steps 10 > gpurun_out/miopen_$i.log 2>&1
  rc=$?; grep RESULT gpurun_out/miopen_$i.log; echo "   exit $rc"
  ok $rc || exit $rc
done <<'CFGS'

MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
CFGS
