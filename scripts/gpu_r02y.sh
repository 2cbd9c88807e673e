#!/bin/bash
# query kernel variants (tuning libraries built with -D flags) vs the default library;
# parity of each library, then timings
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r02z}
mkdir -p $O
lib() { if [ "$1" = default ]; then echo distributedauc_amd/libdauc.so; else echo tuning/libdauc_$1.so; fi; }
for v in default spt4 spt16; do
  DAUC_LIB=$(lib $v) timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
      tests/test_kernels_gpu.py -k "sorted or extreme or auc_counts_large or eval_counts" > $O/tests_$v.log 2>&1 || exit 1
done
for r in 1 2; do
  for v in default spt4 spt16; do
    DAUC_LIB=$(lib $v) timeout -k 10 120 python -u scripts/micro_kernels.py --which aucsort --reps 20 2>/dev/null \
        | sed "s/^{/{\"lib\": \"$v\", /" >> $O/micro.jsonl || exit 1
  done
done
