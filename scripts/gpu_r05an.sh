#!/bin/bash
# round 5: split-K slab sums deferred to the end of the backward pass and batched into one launch
# (DAUC_SLAB_DEFER=1, default) against one sum per layer (DAUC_SLAB_DEFER=0): conv / shadow / R-50
# update tests, training-only runs interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05an}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv1x1_gpu.py tests/test_conv_wgrad_gpu.py \
    tests/test_weight_shadow_gpu.py tests/test_configs_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
for i in 1 2; do
    run sep$i DAUC_SLAB_DEFER=0 || exit $?
    run defer$i DAUC_SLAB_DEFER=1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" \
    --eval-images 0 > $O/trace.log 2>&1 || exit $?
echo done
