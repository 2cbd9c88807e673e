#!/bin/bash
# round 4: the direct count-index build with 256 instead of up to 1024 workgroups (A/B against
# tuning/libdauc_g1024.so), the part probe, the AUC tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/r04q
mkdir -p $D
for n in "27 0.001" "24 0.01"; do
  set -- $n
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/p$1 -o run -- python3 $R/scripts/prof_eval.py $1 $2 5 > $D/p$1.log 2>&1 || exit 1
  DAUC_LIB=$R/tuning/libdauc_g1024.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/o$1 -o run -- python3 $R/scripts/prof_eval.py $1 $2 5 > $D/o$1.log 2>&1 || exit 1
done
cd $R
timeout -k 10 300 python -u scripts/probe_eval_part.py 20 > $D/eval_part_probe.jsonl 2> $D/eval_part_probe.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_auc_cells_gpu.py tests/test_kernels_gpu.py tests/test_auc_slots_gpu.py -q --timeout 300 --timeout-method thread > $D/pytest_auc.log 2>&1
echo "auc tests rc=$?"
