#!/bin/bash
# one GPU call (round 5): the default bench line (kernel, parity sample, host legs incl. the file and
# .gz output legs), then the raw stream's two egress modes at 50 M pairs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.log || exit 1
if [ -n "${EGRESS:-}" ]; then
  timeout -k 10 600 python -u tools/e2e_bench.py --pairs 50000000 --no-ref --null-out --pause 2 --repeat 2 \
     --variants ";FQ_RAW_EGRESS=host" > gpurun_out/e2e_egress.txt 2>&1 || exit 1
fi
