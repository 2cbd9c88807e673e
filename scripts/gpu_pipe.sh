#!/bin/bash
# two-phase (pipelined) query loop: parity of every sort-method test, then the A/B of the
# query pass and the one-call evaluation against the single-phase loop
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pipe
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_auc_cells_gpu.py \
    tests/test_kernels_gpu.py -k "auc or sort or compact" > $O/pytest_sort.log 2>&1 || exit 1
for lib in distributedauc_amd/libdauc.so tuning/libdauc_pu3.so tuning/libdauc_nopipe.so distributedauc_amd/libdauc.so; do
  echo "== $lib" >> $O/micro.jsonl
  DAUC_LIB=$lib timeout -k 10 300 python3 scripts/micro_cells.py 30 1 >> $O/micro.jsonl 2>> $O/micro.err || exit 1
done
