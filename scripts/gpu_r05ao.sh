#!/bin/bash
# round 5: split-K slab sum with plain (cached) loads instead of nontemporal ones
# (tuning/ab/libdauc_slabplain.so, -DDAUC_SLAB_PLAIN) against the shipped build: slab-sum tests,
# training-only runs interleaved, a kernel trace of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05ao}
V=tuning/ab/libdauc_slabplain.so
mkdir -p $O
DAUC_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_conv1x1_gpu.py -x -q -k slab --timeout 120 \
    --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
for i in 1 2 3; do
    run base$i || exit $?
    run plain$i DAUC_LIB=$V || exit $?
done
for v in base plain; do
    L=distributedauc_amd/libdauc.so; [ $v = plain ] && L=$V
    DAUC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o bench -- \
        python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" \
        --eval-images 0 > $O/trace_$v.log 2>&1 || exit $?
done
echo done
