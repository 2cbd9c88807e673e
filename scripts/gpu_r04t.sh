#!/bin/bash
# round 4: the unaligned single-window query with the block-word reads interleaved under the
# previous group's count (ui), + 2 stream groups (ui2): timings and the AUC tests on ui
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04t
mkdir -p $D
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/t0 -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/t0.log 2>&1 || exit 1
for v in un ui ui2 uil; do
  DAUC_LIB=$R/tuning/libdauc_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/$v -o run -- python3 $R/scripts/prof_eval.py 27 0.001 5 > $D/$v.log 2>&1 || exit 1
done
cd $R
DAUC_LIB=$R/tuning/libdauc_ui.so timeout -k 10 600 python -u -m pytest tests/test_auc_cells_gpu.py tests/test_kernels_gpu.py tests/test_integration_gpu.py -k "auc or sort or cells or eval or integration or direct" -q --timeout 300 --timeout-method thread > $D/pytest_ui.log 2>&1
echo "ui tests rc=$?"
