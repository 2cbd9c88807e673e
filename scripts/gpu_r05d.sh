#!/bin/bash
# round 5: BN finalize with grouped loads -- BN tests, the slot-count tweak (two-step tests), then the
# bench's kernel trace (finalize durations vs profiles/r05/step) and a default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_bn_gpu.py tests/test_two_step_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 50 > $O/two_step.jsonl 2> $O/two_step.err || exit $?
cat $O/two_step.jsonl
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/bench_trace.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_step'], d['training_eval']['auc'], d['training_eval']['band'])"
