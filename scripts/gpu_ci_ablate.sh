#!/bin/bash
# count-index query pass ablations (wrong counts by design): 1 no window load, 2 no LDS index,
# 3 neither (stream + key math only); mode 0 = count index
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ciab
mkdir -p $O
for A in 1 2 3; do
  echo "== ablate $A" >> $O/micro.jsonl
  DAUC_LIB=tuning/libdauc_ab$A.so timeout -k 10 300 python3 scripts/micro_cells.py 30 0 >> $O/micro.jsonl 2>> $O/micro.err || exit 1
done
