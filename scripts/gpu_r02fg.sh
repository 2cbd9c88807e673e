#!/bin/bash
set -o pipefail
bash scripts/gpu_r02f.sh && bash scripts/gpu_r02g.sh
