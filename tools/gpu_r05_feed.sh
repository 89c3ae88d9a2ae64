#!/bin/bash
# one GPU call (round 5): raw-stream parity on 1/3/4 engines (GPU), then the host feed ceiling
# (null engines, no GPU) at G = 1, 2, 4, 8 on the box's host cores
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_host_e2e.py tests/test_raw_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
   > gpurun_out/pt_raw.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/host_feed.py --pairs ${PAIRS:-50000000} --engines 1,2,4,8 --workers 16 --repeat 2 \
   > gpurun_out/host_feed.txt 2>&1 || exit 1
