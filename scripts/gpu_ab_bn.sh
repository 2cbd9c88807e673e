#!/bin/bash
# A/B of the BN relu-mask source (read y vs recompute from x): kernel times from rocprofv3, engines pinned
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp DAUC_CONV1X1=gemm
mkdir -p gpurun_out/ab
for v in 0 1; do
  DAUC_BN_MASK_FROM_X=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab -o mask$v -- \
      python -u bench.py --steps 10 --warmup 3 --no-auc --no-surrogate --no-cpu-baseline > gpurun_out/ab/log$v.txt 2>&1
  rc=$?; echo "== mask$v exit $rc"; tail -1 gpurun_out/ab/log$v.txt | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
