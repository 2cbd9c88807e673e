#!/bin/bash
# round 5: BN partial-sum passes, loads in flight per thread: stats 8 / bwd 4 row passes (default)
# against 16 / 4 (u16), 8 / 8 (b8) and 4 / 2 (u4) builds (tuning/ab): BN tests per variant,
# per-shape probe and training-only runs, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05am}
mkdir -p $O
for v in u16 b8; do
    DAUC_LIB=tuning/ab/libdauc_$v.so timeout -k 10 300 python -u -m pytest tests/test_fused_bn_gpu.py -x -q \
        --timeout 120 --timeout-method thread > $O/pytest_bn_$v.log 2>&1
    rc=$?; echo "bn tests $v rc=$rc"; tail -1 $O/pytest_bn_$v.log
    [ $rc -eq 0 ] || exit $rc
done
lib() { [ $1 = base ] && echo distributedauc_amd/libdauc.so || echo tuning/ab/libdauc_$1.so; }
for i in 1 2; do
    for v in base u16 b8 u4; do
        DAUC_LIB=$(lib $v) timeout -k 10 180 python3 scripts/probe_bn.py --tag $v >> $O/probe.jsonl 2>> $O/probe.err || exit $?
    done
done
python3 - $O <<'PY'
import json, sys
for l in open(f"{sys.argv[1]}/probe.jsonl"):
    d = json.loads(l); print(d["tag"], d["shape"], d["fwd_us"], d["bwd_us"], d["bwd_res_us"])
PY
run() {  # name, lib
    timeout -k 10 300 env DAUC_LIB=$2 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$1.json 2> $O/$1.err || return $?
    python3 -c "import json;d=json.load(open('$O/$1.json'));print('$1', round(d['ms_per_step'],3), round(d['value'],1))"
}
for i in 1 2; do
    for v in base u16 b8; do run ${v}$i $(lib $v) || exit $?; done
done
echo done
