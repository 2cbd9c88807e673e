#!/bin/bash
# PMC passes over the bucketed evaluation at 2^27 @ 0.1 %
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04c
mkdir -p $D
P="python3 $R/scripts/prof_eval.py 27 0.001 3"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES -d $D/p1 -o run --output-format csv -- $P > $D/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM -d $D/p2 -o run --output-format csv -- $P > $D/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/p3 -o run --output-format csv -- $P > $D/p3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/p4 -o run --output-format csv -- $P > $D/p4.log 2>&1
