#!/bin/bash
# cell-index search: its parity tests, the A/B timing against the tree, and a kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cells
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_auc_cells_gpu.py \
    > $O/pytest_cells.log 2>&1 || exit 1
timeout -k 10 300 python3 scripts/micro_cells.py 20 > $O/micro_cells.jsonl 2> $O/micro_cells.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o cells -- \
    python3 scripts/micro_cells.py 5 > $O/prof.log 2>&1 || exit 1
DAUC_LIB=tuning/libdauc_cg.so timeout -k 10 300 python3 scripts/micro_cells.py 20 2,1 > $O/micro_cells_group.jsonl 2>> $O/micro_cells.err || exit 1
DAUC_LIB=tuning/libdauc_cg.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_auc_cells_gpu.py > $O/pytest_cells_group.log 2>&1 || exit 1
