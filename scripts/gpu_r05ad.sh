#!/bin/bash
# round 5: BN partial-pass geometry at HEAD: row-block target x threads per workgroup
# (DAUC_BN_ROWBLOCKS, DAUC_BN_PART_THREADS; r01 measured 256 x 512 best), training-only bench runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ad}
mkdir -p $O
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run base1 || exit $?
run rb512_t512 DAUC_BN_ROWBLOCKS=512 || exit $?
run rb256_t1024 DAUC_BN_PART_THREADS=1024 || exit $?
run rb512_t256 DAUC_BN_ROWBLOCKS=512 DAUC_BN_PART_THREADS=256 || exit $?
run rb1024_t256 DAUC_BN_ROWBLOCKS=1024 DAUC_BN_PART_THREADS=256 || exit $?
run base2 || exit $?
echo done
