#!/bin/bash
# conv1x1: the shipped engine plan (measured once) + the TunableOp NaN probe
set -o pipefail
mkdir -p gpurun_out/r02g
export TMPDIR=/tmp
DAUC_CONV1X1_PLANS="" timeout -k 10 300 python -u scripts/gen_conv1x1_plans.py gpurun_out/r02g/conv1x1_plans.json \
    > gpurun_out/r02g/plans.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/probe_tunableop.py profiles/r01/tunableop/results0.csv \
    > gpurun_out/r02g/tunableop_probe.jsonl 2> gpurun_out/r02g/tunableop_probe.err
