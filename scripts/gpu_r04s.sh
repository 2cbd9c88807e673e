#!/bin/bash
# round 4: three-slot pipeline variants and the linear map (timings), then where the waves of the
# count-index query wait (PMC: wait / active-instruction cycle counters) for the product and the
# no-window ablation
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04s
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
for v in up3 up3l uil; do
  DAUC_LIB=$R/tuning/libdauc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/$v -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/$v.log 2>&1 || exit 1
done
C="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $D -o w_t0 -- python3 $R/scripts/prof_eval.py 27 0.001 3 > $D/w_t0.log 2>&1 || exit 1
DAUC_LIB=$R/tuning/libdauc_g24.so timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $D -o w_g24 -- python3 $R/scripts/prof_eval.py 27 0.001 3 > $D/w_g24.log 2>&1 || exit 1
