#!/bin/bash
# round 4: instruction counters of the count-index query (product, unaligned single-window variant,
# no-window ablation) in one PMC pass each
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04u
mkdir -p $D
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $D -o t0 -- python3 $R/scripts/prof_eval.py 27 0.001 3 > $D/t0.log 2>&1 || exit 1
for v in un g24; do
  DAUC_LIB=$R/tuning/libdauc_$v.so timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $D -o $v -- python3 $R/scripts/prof_eval.py 27 0.001 3 > $D/$v.log 2>&1 || exit 1
done
