#!/bin/bash
# round 5: the 3x3 input gradients as forward convolutions (flipped shadow weights) and the
# headline step replayed from a HIP graph with an eager update. Tests first, then short training
# runs interleaved, then a kernel trace of the graph + dgrad configuration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_weight_shadow_gpu.py \
    -q --timeout 200 --timeout-method thread > $O/pytest_new.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest_new.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, shadow, graph
    local name=$1 sh=$2 gr=$3
    timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 --weight-shadow $sh --graph $gr > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1), round(d['roofline']['frac'],3))"
}
run s1_g0 1 0 || exit $?
run s2_g0 2 0 || exit $?
run s2_g1 2 1 || exit $?
run s1_g1 1 1 || exit $?
run s0_g0 0 0 || exit $?
run s2_g1b 2 1 || exit $?
run s2_g0b 2 0 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 --graph 1 > $O/bench_trace.log 2>&1 || exit $?
echo done
