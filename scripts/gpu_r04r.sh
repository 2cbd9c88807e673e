#!/bin/bash
# round 4: the count-index query with VGPR-only counting (no compare -> SGPR -> select chains) and
# +inf pad windows: the AUC / sort / count-index tests, the kernel time, its instruction counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04r
mkdir -p $D
cd $R
timeout -k 10 600 python -u -m pytest tests/test_auc_cells_gpu.py tests/test_kernels_gpu.py tests/test_integration_gpu.py tests/test_auc_slots_gpu.py -q --timeout 300 --timeout-method thread > $D/pytest_auc.log 2>&1
rc=$?
echo "auc tests rc=$rc"
if [ $rc -ge 124 ]; then exit $rc; fi
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t24 -o run -- python3 $R/scripts/prof_eval.py 24 0.01 5 > $D/t24.log 2>&1 || exit 1
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $D -o pmc -- python3 $R/scripts/prof_eval.py 27 0.001 3 > $D/pmc.log 2>&1 || exit 1
