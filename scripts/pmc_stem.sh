#!/bin/bash
# PMC passes over the stem micro-benchmark (scripts/probe_stem.py): issue / wait / LDS / memory
# counters of stem_fwd_kernel and stem_wgrad_kernel (one pass per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_stem}
mkdir -p $O
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_WAVES --output-format csv -d $O -o p1 -- python3 scripts/probe_stem.py 5 > $O/log_p1.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $O -o p2 -- python3 scripts/probe_stem.py 5 > $O/log_p2.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $O -o p3 -- python3 scripts/probe_stem.py 5 > $O/log_p3.txt 2>&1 || exit 1
echo done
