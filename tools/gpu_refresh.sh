#!/bin/bash
# One GPU call: GPU tests, smoke, per-config profiles (kernel trace + PMC traffic at 100 M pairs),
# config bench lines at 100 M pairs, the default bench line.  First failure ends the call.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
fi
for c in ${PROF_CONFIGS:-C3 C4 C5}; do
  ROUND=r02 CONFIG=$c PAIRS=100000000 bash tools/profile_round.sh > gpurun_out/prof_$c.out 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/prof_$c.out; exit 1; }
  echo "profile $c ok"
done
PAIRS=100000000 CONFIGS="${BENCH_CONFIGS:-C2 C4 C5}" bash tools/configs_bench.sh > gpurun_out/configs_100M.txt 2>&1 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
grep '"metric"' gpurun_out/bench.log | tail -n 1
