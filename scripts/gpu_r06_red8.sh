#!/bin/bash
# round 6: the query pass's end-of-kernel reduction through 8 group lines (query_ci_kernel's red8)
# instead of 3-4 atomics per workgroup on the record's line -- the AUC GPU tests, then the
# per-rank probe interleaving the product library with the previous commit's build
# (tuning/libdauc_base.so), and the ablation probe (tuning build) for the attribution.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06red8
mkdir -p $O
scripts/gpu_step.sh r06red8/pytest_auc 480 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_two_step_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py tests/test_auc_fuzz_gpu.py \
    tests/test_kernels_gpu.py -k "auc or eval or two_step or count or split or pair or sort or fuzz"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 40 --base=tuning/libdauc_base.so > $O/probe_base.jsonl 2> $O/probe_base.err; rc=$?
echo "probe rc=$rc"; tail -2 $O/probe_base.err
[ $rc -eq 0 ] || exit $rc
for abl in 0 3; do
  DAUC_QUERY_ABL=$abl timeout -k 10 120 python -u scripts/probe_query_abl.py 40 >> $O/abl.jsonl 2>> $O/abl.err || exit $?
done
echo done
