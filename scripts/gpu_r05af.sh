#!/bin/bash
# round 5: the 1x1 engine plan re-measured with TunableOp's checked GEMM selections in the loop
# (scripts/tune_joint.py), then training-only runs: shipped plan + shipped selections against the
# new plan + new selections, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05af}
mkdir -p $O
DAUC_CONV1X1_PLANS= timeout -k 10 900 python -u scripts/tune_joint.py $O/plans_joint.json $O/tunableop_joint.csv > $O/tune.log 2>&1 || exit $?
tail -3 $O/tune.log
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run ship1 || exit $?
run joint1 DAUC_CONV1X1_PLANS=$O/plans_joint.json DAUC_TUNABLEOP=$O/tunableop_joint.csv || exit $?
run ship2 || exit $?
run joint2 DAUC_CONV1X1_PLANS=$O/plans_joint.json DAUC_TUNABLEOP=$O/tunableop_joint.csv || exit $?
echo done
