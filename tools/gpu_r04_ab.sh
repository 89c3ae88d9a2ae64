#!/bin/bash
# one GPU call (round 4): optional opcost2 microbench, A/B of build/alt variants (tools/ab.sh),
# then the engine parity tests on the default build.  ALTS="base pl" CONFIGS="C3 C4" TESTS="..."
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ -n "${OPCOST:-}" ]; then timeout -k 10 200 ./build/micro/opcost2 > gpurun_out/opcost2.txt 2>&1 || exit 1; fi
if [ -n "${SEL:-}" ]; then timeout -k 10 200 ./build/micro/sel > gpurun_out/sel.txt 2>&1 || exit 1; fi
if [ -n "${ALTS:-}" ]; then
  ALTS="$ALTS" CONFIGS="${CONFIGS:-C3}" REPS=${REPS:-2} bash tools/ab.sh > gpurun_out/ab.txt 2>&1 || exit 1
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1 || exit 1
fi
exit 0
