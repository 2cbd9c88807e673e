#!/bin/bash
# round 5: the window wgrad kernel with 32-bit LDS and global offsets (the 64-bit address math was
# most of its loop VALU). Tests, then training-only runs against the previous build
# (tuning/ab/libdauc_win1.so) interleaved, then a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_wgrad_gpu.py tests/test_weight_shadow_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest_wgrad.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; tail -2 $O/pytest_wgrad.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run prev1 DAUC_LIB=tuning/ab/libdauc_win1.so || exit $?
run new1 || exit $?
run prev2 DAUC_LIB=tuning/ab/libdauc_win1.so || exit $?
run new2 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/bench_trace.log 2>&1 || exit $?
echo done
