#!/bin/bash
# round 5: TunableOp selections for the bench's hipBLASLt GEMMs (numerically checked against the
# default solution), then training-only runs with the default solutions and with the selections,
# interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ae}
mkdir -p $O
timeout -k 10 900 python -u scripts/tune_gemms.py $O/tunableop.csv > $O/tune.log 2>&1 || exit $?
tail -2 $O/tune.log; ls -la $O/tunableop*.csv
F=$(ls $O/tunableop*.csv | head -1)
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run def1 || exit $?
run tuned1 DAUC_TUNABLEOP=$F || exit $?
run def2 || exit $?
run tuned2 DAUC_TUNABLEOP=$F || exit $?
echo done
