#!/bin/bash
# round 4: the query pass's PMC counters (instruction mix, LDS waits) and kernel durations at
# 2^27 / 2^24 of the one-call evaluation (scripts/prof_eval.py; scripts/query_valu.py -> profiles/query_valu.json)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_r04q
mkdir -p $O
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O -o valu -- \
    python3 scripts/prof_eval.py 27 0.001 3 > $O/log_valu.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv \
    -d $O -o valu24 -- python3 scripts/prof_eval.py 24 0.01 3 > $O/log_valu24.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
    SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES --output-format csv -d $O -o lds -- \
    python3 scripts/prof_eval.py 27 0.001 3 > $O/log_lds.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- \
    python3 scripts/prof_eval.py 27 0.001 5 > $O/log_trace.txt 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace24 -- \
    python3 scripts/prof_eval.py 24 0.01 5 > $O/log_trace24.txt 2>&1 || exit 1
