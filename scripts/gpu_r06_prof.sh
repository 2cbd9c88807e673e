#!/bin/bash
# round-6 evidence, profiles: the bench's kernel trace (the line's command, shortened), PMC HBM traffic
# of the roofline kernels (update, loss: micro_kernels; the evaluation's query: prof_eval 2^27), and
# the query pass's instruction mix / LDS counters / durations (-> scripts/query_valu.py). One counter
# group per pass, each under its own limit; a failing pass ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06prof
mkdir -p $O
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_trace.json 2> $O/bench_trace.err || exit $?
echo "bench trace done"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc -o pmc_$c -- \
      python3 scripts/micro_kernels.py --which update,surrogate --variants 0 --reps 5 > $O/log_$c.txt 2>&1 || exit $?
  timeout -k 10 -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc -o pmcq_$c -- \
      python3 scripts/prof_eval.py 27 0.001 3 > $O/logq_$c.txt 2>&1 || exit $?
  echo "pmc $c done"
done
Q=$O/query
mkdir -p $Q
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $Q -o valu27 -- \
    python3 scripts/prof_eval.py 27 0.001 3 > $Q/log_valu27.txt 2>&1 || exit $?
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --output-format csv \
    -d $Q -o valu24 -- python3 scripts/prof_eval.py 24 0.01 3 > $Q/log_valu24.txt 2>&1 || exit $?
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
    SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES --output-format csv -d $Q -o lds27 -- \
    python3 scripts/prof_eval.py 27 0.001 3 > $Q/log_lds27.txt 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $Q -o trace27 -- \
    python3 scripts/prof_eval.py 27 0.001 5 > $Q/log_trace27.txt 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $Q -o trace24 -- \
    python3 scripts/prof_eval.py 24 0.01 5 > $Q/log_trace24.txt 2>&1 || exit $?
echo "query pmc done"
