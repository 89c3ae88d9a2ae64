#!/bin/bash
# raw-stream ingest (pread staging): golden e2e parity incl. the small-window stress test, then the
# 50 M-pair e2e (raw vs text packs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_host_e2e.py tests/test_text_gpu.py \
    -m gpu > gpurun_out/t_raw2.log 2>&1 || { tail -40 gpurun_out/t_raw2.log; exit 1; }
tail -2 gpurun_out/t_raw2.log
VARIANTS="${VARIANTS- ;FQ_RAW_MODE=0}" bash tools/gpu_e2e_var.sh
