#!/bin/bash
# round 3: where the count-index query waits on the memory side (2^27 @ 0.1 %): L1->L2 requests and
# their latency, L2 hit rate and busy, TA/TD busy, vector-memory instruction levels. One --pmc pass
# per counter group (the per-block limits), each under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_mem
mkdir -p $O
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o kt -- python3 scripts/probe_query.py 27 0.001 3 > $O/log_kt.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $O -o p1 -- python3 scripts/probe_query.py 27 0.001 3 > $O/log_p1.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_BUSY_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $O -o p2 -- python3 scripts/probe_query.py 27 0.001 3 > $O/log_p2.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_WAVES TD_TC_STALL_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum --output-format csv -d $O -o p3 -- python3 scripts/probe_query.py 27 0.001 3 > $O/log_p3.txt 2>&1 || exit 1
