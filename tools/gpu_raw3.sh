#!/bin/bash
# raw streams: engine-level tests, golden e2e (incl. small windows), 10 M-pair e2e diagnostics
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_raw_gpu.py \
    -m gpu > gpurun_out/t_raw3a.log 2>&1 || { tail -60 gpurun_out/t_raw3a.log; exit 1; }
tail -2 gpurun_out/t_raw3a.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_host_e2e.py \
    -m gpu > gpurun_out/t_raw3b.log 2>&1 || { tail -40 gpurun_out/t_raw3b.log; exit 1; }
tail -2 gpurun_out/t_raw3b.log
PAIRS=${PAIRS:-10000000} VARIANTS="${VARIANTS- }" bash tools/gpu_e2e_var.sh
