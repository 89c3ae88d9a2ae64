#!/bin/bash
# one GPU call (round 6): the full GPU test suite on the in-tree build, then the host feed ceiling
# with null engines on the box's host cores (tools/host_feed.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 ${SUITE_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
     > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "${FEED:-0}" = 1 ]; then
  timeout -k 10 600 python -u tools/host_feed.py --pairs ${FEED_PAIRS:-50000000} --engines 1,2,4,8 --workers ${FEED_W:-16} \
     --repeat 2 > gpurun_out/host_feed.txt 2>&1 || { tail -20 gpurun_out/host_feed.txt; exit 1; }
  cat gpurun_out/host_feed.txt | cut -c1-220
fi
