#!/bin/bash
# round 6: PMC counters of the distinct-key query pass (bf16-rounded 2^27 @ 0.1 %, the one-call
# evaluation's verdict-2 path): instruction mix + LDS counters, then HBM traffic (FETCH_SIZE, WRITE_SIZE:
# separate passes), each pass under its own limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06dkpmc
mkdir -p $O
timeout -k 10 -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $O -o sq -- \
    python3 scripts/probe_eval_ties.py 3 --only bf16 27 > $O/log_sq.txt 2>&1 &&
timeout -k 10 -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O -o fetch -- \
    python3 scripts/probe_eval_ties.py 3 --only bf16 27 > $O/log_fetch.txt 2>&1 &&
timeout -k 10 -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O -o write -- \
    python3 scripts/probe_eval_ties.py 3 --only bf16 27 > $O/log_write.txt 2>&1 &&
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- \
    python3 scripts/probe_eval_ties.py 3 --only bf16 27 > $O/log_trace.txt 2>&1 && echo done
