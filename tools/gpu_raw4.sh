#!/bin/bash
# raw streams: engine tests + golden e2e, then 50 M-pair e2e variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_raw_gpu.py tests/test_host_e2e.py \
    -m gpu > gpurun_out/t_raw4.log 2>&1 || { tail -40 gpurun_out/t_raw4.log; exit 1; }
tail -2 gpurun_out/t_raw4.log
PAIRS=${PAIRS:-50000000} VARIANTS="${VARIANTS- ;FQ_RAW_MODE=0}" REPEAT=${REPEAT:-1} bash tools/gpu_e2e_var.sh
