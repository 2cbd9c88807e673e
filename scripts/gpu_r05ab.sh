#!/bin/bash
# round 5: window staging through buffer descriptors (range-checked zeros) and immediate tap offsets; every form timed, and a
# cost-model choice of the layout. wgrad tests (every form), micro-benchmark per form, training-only
# runs against the previous build ($PREV) interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05x}
PREV=${PREV:-tuning/ab/libdauc_sh2.so}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_conv_wgrad_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest_wgrad.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; tail -2 $O/pytest_wgrad.log
[ $rc -eq 0 ] || exit $rc
for f in 1 4 5; do
    timeout -k 10 120 python3 scripts/probe_wgrad.py 20 $f >> $O/probe.jsonl 2>> $O/probe.err || exit $?
done
timeout -k 10 120 python3 scripts/probe_wgrad.py 20 >> $O/probe.jsonl 2>> $O/probe.err || exit $?
DAUC_LIB=$PREV timeout -k 10 120 python3 scripts/probe_wgrad.py 20 > $O/probe_prev.jsonl 2>> $O/probe.err || exit $?
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for l in list(open(f"{o}/probe.jsonl")) + [l.replace('"form": "auto"', '"form": "prev"') for l in open(f"{o}/probe_prev.jsonl")]:
    d = json.loads(l); print(d["form"], d["C"], d["H"], d["stride"], round(d["us_per_call"], 1))
PY
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run prev1 DAUC_LIB=$PREV || exit $?
run new1 || exit $?
run prev2 DAUC_LIB=$PREV || exit $?
run new2 || exit $?
echo done
