#!/bin/bash
# query kernel: per-kernel times, then SQ counters (one pass, 8 SQ counters)
set -o pipefail
mkdir -p gpurun_out/r02c
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02c/trace -o run -- python3 scripts/probe_query.py 27 0.001 5 \
    > gpurun_out/r02c/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU -d gpurun_out/r02c/pmc1 -o run -- python3 scripts/probe_query.py 27 0.001 2 \
    > gpurun_out/r02c/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS \
    SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD -d gpurun_out/r02c/pmc2 -o run -- python3 scripts/probe_query.py 27 0.001 2 \
    > gpurun_out/r02c/pmc2.log 2>&1
