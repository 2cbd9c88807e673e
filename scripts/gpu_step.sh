#!/bin/bash
# Run one GPU step under its own time limit; record its exit status.
# Usage: scripts/gpu_step.sh NAME SECONDS cmd...   (output -> gpurun_out/NAME.log)
# Exit 0/1 (pass / ordinary test failure) lets the caller continue; anything else
# (timeout 124/137, abort 134, segfault 139, ...) must end the GPU call.
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "== $name: $*" 
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name exit $rc"
tail -n 25 "gpurun_out/$name.log"
exit $rc
