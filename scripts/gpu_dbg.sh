#!/bin/bash
timeout -k 10 300 python -u -m pytest -x -v --timeout 250 --timeout-method thread tests/test_main_gpu.py::test_main_split_scoring_world2 > gpurun_out/pytest_dbg.log 2>&1
