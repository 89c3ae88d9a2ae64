#!/bin/bash
# Round-3 profiles of the final build: C3 kernel trace + PMC traffic (profile_round.sh), SQ issue/LDS
# counters of C3, and the 100 M-pair bench lines of C2, C4, C5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ "${SKIP_ROUND:-0}" = 1 ] || ROUND=r03 CONFIG=C3 bash tools/profile_round.sh > gpurun_out/profile_round_C3.log 2>&1 || { tail -5 gpurun_out/profile_round_C3.log; exit 1; }
[ "${SKIP_ROUND:-0}" = 1 ] || tail -3 gpurun_out/profile_round_C3.log
CONFIGS=C3 bash tools/pmc_sq.sh > gpurun_out/pmc_sq_C3.log 2>&1 || { tail -5 gpurun_out/pmc_sq_C3.log; exit 1; }
for c in C2 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --pairs 100000000 --steps 5 --warmup 1 --no-cpu-baseline --engine-pairs 0 --sample-pairs 0 > gpurun_out/b100_$c.log 2>&1 || exit 1
  grep '"metric"' gpurun_out/b100_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"
done
