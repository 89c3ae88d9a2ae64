#!/bin/bash
# one GPU call (round 5): raw-stream parity (engine + binary), then e2e C3 and C4 at 50 M pairs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_raw_gpu.py tests/test_host_e2e.py tests/test_text_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
   > gpurun_out/pt_exact.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/e2e_bench.py --pairs 50000000 --no-ref --null-out --pause 2 --repeat 3 > gpurun_out/e2e_exact_c3.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/e2e_bench.py --pairs 50000000 --no-ref --null-out --pause 2 --repeat 3 --config C4 > gpurun_out/e2e_exact_c4.txt 2>&1 || exit 1
