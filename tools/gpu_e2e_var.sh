#!/bin/bash
# e2e variants on one generated input: VARIANTS (';'-separated tool options), PAIRS, WL
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 ${TMO:-600} python -u tools/e2e_bench.py --pairs ${PAIRS:-50000000} --null-out --workers-list ${WL:-16} \
  --variants "${VARIANTS:-}" --repeat ${REPEAT:-1} > gpurun_out/e2e_var.txt 2>&1 || { tail -5 gpurun_out/e2e_var.txt; exit 1; }
cat gpurun_out/e2e_var.txt
