#!/bin/bash
# one GPU call (round 5): kernel A/B of build/alt variants, then the engine parity tests on one variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
ALTS="${ALTS:-A B}" CONFIGS="${CONFIGS:-C3 C4}" REPS=${REPS:-2} bash tools/ab.sh > gpurun_out/ab.txt 2>&1 || exit 1
if [ -n "${TEST_LIB:-}" ]; then
  FQ_ENGINE_LIB=$PWD/build/alt/lib_$TEST_LIB.so timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_engine_gpu.py} -x -q \
     --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1 || exit 1
fi
