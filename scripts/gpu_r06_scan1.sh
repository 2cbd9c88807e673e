#!/bin/bash
# round 6: the one-call slotted count pass (direct_count_kernel<true>) with one workgroup scan: the key
# total from the compaction's P, the used buckets by ballots -- the AUC GPU tests, then the probe interleaving
# the product library with the previous commit (tuning/libdauc_head.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06scan1
mkdir -p $O
scripts/gpu_step.sh r06scan1/pytest_auc 480 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    tests/test_two_step_gpu.py tests/test_auc_cells_gpu.py tests/test_integration_gpu.py tests/test_auc_fuzz_gpu.py tests/test_auc_ties_gpu.py \
    tests/test_kernels_gpu.py -k "auc or eval or two_step or count or split or pair or sort or fuzz"; rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 40 --base=tuning/libdauc_head.so > $O/probe_base.jsonl 2> $O/probe_base.err; rc=$?
echo "probe rc=$rc"; tail -2 $O/probe_base.err
exit $rc
