#!/bin/bash
# round 5: PMC passes over the stem and 3x3 weight-gradient micro-benchmarks (scripts/probe_stem.py,
# scripts/probe_wgrad.py): HBM traffic (FETCH_SIZE, WRITE_SIZE; separate passes) and the wgrad
# kernel's issue / wait counters. One counter group per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r05_convs}
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O -o stem_$c -- python3 scripts/probe_stem.py 3 > $O/log_stem_$c.txt 2>&1 || exit 1
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O -o wgrad_$c -- python3 scripts/probe_wgrad.py 3 > $O/log_wgrad_$c.txt 2>&1 || exit 1
done
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAVES --output-format csv -d $O -o wgrad_sq1 -- python3 scripts/probe_wgrad.py 3 > $O/log_wgrad_sq1.txt 2>&1 || exit 1
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $O -o wgrad_sq2 -- python3 scripts/probe_wgrad.py 3 > $O/log_wgrad_sq2.txt 2>&1 || exit 1
echo done
