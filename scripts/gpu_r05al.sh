#!/bin/bash
# round 5: BN partial-sum passes with the interleaved row-group walk (DAUC_BN_INTERLEAVE=1) against
# the contiguous row blocks: BN tests under the interleaved walk, per-shape probe and training-only
# runs, interleaved A/B in separate processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r05al}
mkdir -p $O
DAUC_BN_INTERLEAVE=1 timeout -k 10 300 python -u -m pytest tests/test_fused_bn_gpu.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest_bn.log 2>&1
rc=$?; echo "bn tests rc=$rc"; tail -2 $O/pytest_bn.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
    for v in 0 1; do
        DAUC_BN_INTERLEAVE=$v timeout -k 10 180 python3 scripts/probe_bn.py --tag r$i >> $O/probe.jsonl 2>> $O/probe.err || exit $?
    done
done
python3 - $O <<'PY'
import json, sys
for l in open(f"{sys.argv[1]}/probe.jsonl"):
    d = json.loads(l); print(d["tag"], d["interleave"], d["shape"], d["fwd_us"], d["bwd_us"], d["bwd_res_us"])
PY
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-auc --no-surrogate \
        --r18-steps 0 --sweep-I "" --eval-images 0 > $O/$name.json 2> $O/$name.err || return $?
    python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name', round(d['ms_per_step'],3), round(d['value'],1))"
}
run contig1 DAUC_BN_INTERLEAVE=0 || exit $?
run inter1 DAUC_BN_INTERLEAVE=1 || exit $?
run contig2 DAUC_BN_INTERLEAVE=0 || exit $?
run inter2 DAUC_BN_INTERLEAVE=1 || exit $?
echo done
