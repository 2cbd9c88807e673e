#!/bin/bash
# round 5: strided pick / strided add / broadcast copies on csrc/strided.hip (downsample backward,
# average-pool gradient). Their tests and the 1x1 / pool / step tests, two training-only bench
# runs, a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ag}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_strided_gpu.py tests/test_conv1x1_gpu.py tests/test_maxpool_gpu.py tests/test_weight_shadow_gpu.py -x -q --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run new1 || exit $?
run new2 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/bench_trace.log 2>&1 || exit $?
echo done
