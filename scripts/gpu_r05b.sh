#!/bin/bash
# round 5: the loss-timeout status test, the two-step per-rank probe (+ its kernel trace), the
# default bench line with the in-training AUC band, and the bench's kernel trace (step breakdown)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u -m pytest "tests/test_kernels_gpu.py::test_surrogate_timeout_reports_status" tests/test_two_step_gpu.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u scripts/probe_two_step.py 50 > $O/two_step.jsonl 2> $O/two_step.err || exit $?
cat $O/two_step.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace2 -o two_step -- python3 scripts/probe_two_step.py 20 --trace > $O/two_step_trace.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || exit $?
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['training_eval']['auc'], d['training_eval']['band'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-auc --no-surrogate --r18-steps 0 --sweep-I "" --eval-images 0 > $O/bench_trace.log 2>&1 || exit $?
exit $rc
