#!/bin/bash
# round 5: the 1x1 input gradient as a forward convolution with W^T ("fconv" engine). Tests, a
# fresh engine plan measured with all three dgrad engines, then the shipped plan vs the new one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv1x1_gpu.py -q --timeout 500 --timeout-method thread \
    > $O/pytest_conv1x1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest_conv1x1.log
[ $rc -eq 0 ] || exit $rc
DAUC_CONV1X1_PLANS= timeout -k 10 400 python -u scripts/gen_conv1x1_plans.py $O/plans_new.json > $O/gen_plans.log 2>&1 || exit $?
tail -2 $O/gen_plans.log
run() {  # name, plans
    local name=$1 pl=$2
    DAUC_CONV1X1_PLANS=$pl timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc \
        --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run old1 distributedauc_amd/conv1x1_plans.json || exit $?
run new1 $O/plans_new.json || exit $?
run old2 distributedauc_amd/conv1x1_plans.json || exit $?
run new2 $O/plans_new.json || exit $?
python3 - <<PY
import json
a = json.load(open("distributedauc_amd/conv1x1_plans.json"))["plans"]
b = json.load(open("$O/plans_new.json"))["plans"]
for k in sorted(set(a) | set(b)):
    if a.get(k) != b.get(k):
        print(k, a.get(k), "->", b.get(k))
PY
echo done
