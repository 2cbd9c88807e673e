#!/bin/bash
# round 5: the 7x7 stem on csrc/conv_stem.hip (forward + weight gradient). Stem parity tests, the
# weight-shadow step tests, micro-benchmark against MIOpen, two training-only bench runs, a
# kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_conv_stem_gpu.py -x -v --timeout 240 --timeout-method thread \
    > $O/pytest_stem.log 2>&1
rc=$?; echo "stem tests rc=$rc"; tail -3 $O/pytest_stem.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/probe_stem.py 20 > $O/probe_stem.jsonl 2> $O/probe_stem.err || exit $?
cat $O/probe_stem.jsonl
timeout -k 10 400 python -u -m pytest tests/test_weight_shadow_gpu.py -x -q --timeout 240 --timeout-method thread \
    > $O/pytest_shadow.log 2>&1
rc=$?; echo "shadow tests rc=$rc"; tail -2 $O/pytest_shadow.log
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
