#!/bin/bash
# one GPU call (round 6): kernel A/B of build/alt variants (tools/ab_build.sh) over CONFIGS, optionally
# with explicit adapters (ADAPTERS=1: C3b), then optional tests on the in-tree engine (TESTS=...).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
if [ -n "${ALTS:-}" ]; then
  ALTS="$ALTS" CONFIGS="${CONFIGS:-C3}" REPS=${REPS:-2} bash tools/ab.sh > gpurun_out/ab.txt 2>&1 || exit 1
  if [ -n "${ALTS_B:-}" ]; then  # a second A/B on C3b (explicit adapter sequences)
    ADAPTERS=1 ALTS="$ALTS_B" CONFIGS="C3" REPS=${REPS:-2} bash tools/ab.sh > gpurun_out/ab_c3b.txt 2>&1 || exit 1
  fi
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q -m gpu --timeout 300 --timeout-method thread \
     > gpurun_out/pt.log 2>&1 || exit 1
fi
