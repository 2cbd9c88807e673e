#!/bin/bash
# count index: every sort-method parity test (mode 0 is the count index where it fits), then the
# A/B of the query pass and the one-call evaluation against the tree, and a kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ci
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_auc_cells_gpu.py \
    > $O/pytest_cells.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
    -k "auc or sort or compact" > $O/pytest_sort.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/micro_cells.py 30 1,0 > $O/micro_ci.jsonl 2> $O/micro.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ci -- \
    python3 scripts/micro_cells.py 5 0 > $O/prof.log 2>&1 || exit 1
DAUC_LIB=tuning/libdauc_ciu1.so timeout -k 10 300 python3 scripts/micro_cells.py 30 0 > $O/micro_ci_u1.jsonl 2>> $O/micro.err || exit 1
