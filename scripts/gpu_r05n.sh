#!/bin/bash
# round 5: where the 3x3 weight-gradient kernel spends its cycles: event times per shape, then
# rocprofv3 PMC passes (one pass each, counters within the per-block limits).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 120 python3 scripts/probe_wgrad.py 20 > $O/probe.jsonl 2> $O/probe.err || exit $?
cat $O/probe.jsonl
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $O/pmc1 -o p -- python3 scripts/probe_wgrad.py 3 > $O/pmc1.log 2>&1 || exit $?
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAVES --output-format csv -d $O/pmc2 -o p -- python3 scripts/probe_wgrad.py 3 > $O/pmc2.log 2>&1 || exit $?
echo done
