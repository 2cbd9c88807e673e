#!/bin/bash
# round 5: the BN ReLU mask -- BN tests first, then the whole GPU suite, the bench's kernel trace and
# a default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_bn_gpu.py -q --timeout 200 --timeout-method thread > $O/pytest_bn.log 2>&1
rc=$?; echo "bn tests rc=$rc"; tail -3 $O/pytest_bn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/bench_trace.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d['training_eval']['auc'], d['training_eval']['band']['in_band'])"
DAUC_BENCH_RECORD_DIR=$O timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 $O/pytest_gpu.log
exit $rc
