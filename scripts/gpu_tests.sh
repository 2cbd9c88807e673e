#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
scripts/gpu_step.sh pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
