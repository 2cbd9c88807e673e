#!/bin/bash
# where the labeled query kernel waits: LDS bank conflicts and wait cycles (2^27 @ 0.1 %)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_lds
mkdir -p $O
timeout -k 10 -s KILL 90 rocprofv3 -L > $O/avail.txt 2>&1 || true
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
    SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $O -o lds -- \
    python3 scripts/probe_query.py 27 0.001 3 > $O/log_lds.txt 2>&1 || exit 1
