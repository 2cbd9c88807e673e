#!/bin/bash
# round 5: BN finalize (batched partial loads + pairwise tree), the stem max-pool's unrolled k=3
# kernels, the bf16 weight shadow, and the BN partial passes' row blocks.
# Tests of the three first, then short bench runs (training only) interleaved: head = the
# previous library (tuning/ab/libdauc_head.so) without the shadow, new = this tree's.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_bn_gpu.py tests/test_maxpool_gpu.py tests/test_weight_shadow_gpu.py \
    -q --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest_new.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, shadow, env...
    local name=$1 sh=$2; shift 2
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 --weight-shadow $sh > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run head1 0 DAUC_LIB=tuning/ab/libdauc_head.so || exit $?
run new_s0 0 || exit $?
run new_s1 1 || exit $?
run new_s1_rb512 1 DAUC_BN_ROWBLOCKS=512 || exit $?
run new_s1_rb512_t256 1 DAUC_BN_ROWBLOCKS=512 DAUC_BN_PART_THREADS=256 || exit $?
run new_s1_rb1024_t256 1 DAUC_BN_ROWBLOCKS=1024 DAUC_BN_PART_THREADS=256 || exit $?
run new_s1_rb512_t1024 1 DAUC_BN_ROWBLOCKS=512 DAUC_BN_PART_THREADS=1024 || exit $?
run new_s1b 1 || exit $?
run head2 0 DAUC_LIB=tuning/ab/libdauc_head.so || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/bench_trace.log 2>&1 || exit $?
echo done
