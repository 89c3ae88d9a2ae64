#!/bin/bash
# one GPU call: A/B of build/alt variants, then ablations and the engine parity tests on the default build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
ALTS="${ALTS:-G H}" CONFIGS="${CONFIGS:-C4 C5}" REPS=${REPS:-2} bash tools/ab.sh > gpurun_out/ab.txt 2>&1 || exit 1
if [ -n "${ABL_CONFIGS:-}" ]; then CONFIGS="$ABL_CONFIGS" bash tools/ablate_cfg.sh > gpurun_out/abl.txt 2>&1 || exit 1; fi
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_engine_gpu.py tests/test_fullsize_gpu.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1
