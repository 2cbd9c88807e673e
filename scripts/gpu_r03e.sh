#!/bin/bash
# eval fix + split in-training scoring (world 2 on cuda:0) + bench's training-eval leg; query-kernel
# ablation timings and PMC passes on the 2^27 evaluation
set -o pipefail
mkdir -p gpurun_out/pmc
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_main_gpu.py \
    "tests/test_kernels_gpu.py::test_auc_eval_counts_one_call" tests/test_kernels_gpu.py::test_auc_eval_enqueue_records \
    > gpurun_out/pytest_e.log 2>&1 &&
timeout -k 10 400 python -u bench.py --no-auc --no-surrogate --no-cpu-baseline --sweep-I "" --r18-steps 0 --steps 10 \
    > gpurun_out/bench_e.log 2>&1 &&
for a in 1 2 3; do
  DAUC_LIB=tuning/libdauc_ab$a.so timeout -k 10 120 python -u scripts/ab_eval.py 10 ab$a >> gpurun_out/ablate.log 2>&1 || exit 1
done &&
timeout -k 10 120 python -u scripts/ab_eval.py 10 product >> gpurun_out/ablate.log 2>&1 &&
(rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true) &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS \
    -d gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 scripts/pmc_eval.py 5 > gpurun_out/pmc/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM \
    -d gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 scripts/pmc_eval.py 5 > gpurun_out/pmc/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum \
    -d gpurun_out/pmc/p3 -o p3 --output-format csv -- python3 scripts/pmc_eval.py 5 > gpurun_out/pmc/p3.log 2>&1
