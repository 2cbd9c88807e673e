#!/bin/bash
# HBM traffic of the roofline kernels from PMC counters: one counter group per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), kernel trace only.
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
R=${ROUND:-r01}
mkdir -p gpurun_out/pmc_$R
for c in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $c"
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_$R -o pmc_$c -- \
      python -u scripts/micro_kernels.py --which update,surrogate --variants 0 --reps 5 \
      > gpurun_out/pmc_$R/log_$c.txt 2>&1
  rc=$?; echo "== pmc $c exit $rc"; tail -3 gpurun_out/pmc_$R/log_$c.txt
  [ $rc -eq 0 ] || exit $rc
done
