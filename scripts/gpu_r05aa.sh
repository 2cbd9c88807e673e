#!/bin/bash
# round 5: the strided 1x1 downsample's backward as GEMMs on x[:, :, ::2, ::2] (forward unchanged on
# the convolution solvers). 1x1 + step tests, the engine plan extended to the new backward shapes
# (existing entries kept), training-only runs against the MIOpen backward
# (DAUC_DOWNSAMPLE_BWD=miopen) interleaved, with the extended plan.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05aa}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv1x1_gpu.py tests/test_weight_shadow_gpu.py tests/test_conv_wgrad_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
cp distributedauc_amd/conv1x1_plans.json $O/plans_in.json
DAUC_CONV1X1_PLANS=$O/plans_in.json timeout -k 10 400 python -u scripts/gen_conv1x1_plans.py $O/plans_new.json > $O/gen_plans.log 2>&1 || exit $?
tail -1 $O/gen_plans.log
run() {  # name, env...
    local name=$1; shift
    env DAUC_CONV1X1_PLANS=$O/plans_new.json "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run prev1 DAUC_DOWNSAMPLE_BWD=miopen || exit $?
run new1 || exit $?
run prev2 DAUC_DOWNSAMPLE_BWD=miopen || exit $?
run new2 || exit $?
echo done
