#!/bin/bash
# round 4: window-load ablations of the count-index query (wrong counts by design): g24 = no
# gathers and no window loads at all, g32 = the second window from registers
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04v
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
for v in g24 g32 un; do
  DAUC_LIB=$R/tuning/libdauc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/$v -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/$v.log 2>&1 || exit 1
done
cd $R
DAUC_LIB=$R/tuning/libdauc_un.so timeout -k 10 600 python -u -m pytest tests/test_auc_cells_gpu.py tests/test_kernels_gpu.py tests/test_integration_gpu.py -k "auc or sort or cells or eval or integration or direct" -q --timeout 300 --timeout-method thread > $D/pytest_un.log 2>&1
echo "un tests rc=$?"
