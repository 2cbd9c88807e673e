#!/bin/bash
# round 5: the 3x3 weight gradient as a hand-written MFMA kernel (csrc/conv_wgrad.hip). Its tests
# first (the transposing read's lane map, fp64 parity, the bench shapes), the shadow/step tests,
# then short training-only runs (--weight-shadow 2 = MIOpen wgrad, 3 = the HIP kernel) interleaved
# and a kernel trace of the new default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_wgrad_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_wgrad.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; tail -15 $O/pytest_wgrad.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_weight_shadow_gpu.py tests/test_fused_bn_gpu.py -q --timeout 240 \
    --timeout-method thread > $O/pytest_shadow.log 2>&1
rc=$?; echo "shadow tests rc=$rc"; tail -3 $O/pytest_shadow.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, shadow mode
    local name=$1 sh=$2
    timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 --weight-shadow $sh > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run s2a 2 || exit $?
run s3a 3 || exit $?
run s2b 2 || exit $?
run s3b 3 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/bench_trace.log 2>&1 || exit $?
echo done
