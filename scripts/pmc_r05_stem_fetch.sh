#!/bin/bash
# round 5: the stem kernels' HBM fetch with XCD-aware task ranges (one FETCH_SIZE pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r05_stem_fetch}
mkdir -p $O
timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O -o stem_FETCH_SIZE -- python3 scripts/probe_stem.py 3 > $O/log.txt 2>&1 || exit 1
echo done
