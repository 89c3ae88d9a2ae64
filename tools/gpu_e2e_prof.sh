#!/bin/bash
# e2e stage profile: the fqtool binary at -w 1/4/8/16 on 10 M pairs, then -w 16 on 50 M pairs
# (outputs to /dev/null, as bench.py's e2e leg)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
df -h /tmp | tail -1
timeout -k 10 400 python -u tools/e2e_bench.py --pairs 10000000 --null-out --workers-list ${WL:-1,4,8,16} > gpurun_out/e2e_prof_10M.txt 2>&1 || { tail -5 gpurun_out/e2e_prof_10M.txt; exit 1; }
cat gpurun_out/e2e_prof_10M.txt
if [ "${BIG:-1}" = 1 ]; then
timeout -k 10 500 python -u tools/e2e_bench.py --pairs 50000000 --null-out --repeat 2 > gpurun_out/e2e_prof_50M.txt 2>&1 || { tail -5 gpurun_out/e2e_prof_50M.txt; exit 1; }
cat gpurun_out/e2e_prof_50M.txt
fi
