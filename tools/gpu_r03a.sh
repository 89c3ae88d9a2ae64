#!/bin/bash
# round-3 GPU step: staging A/B, engine/e2e/kmer parity, detection stage timing, e2e tool timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
ALTS="ovx2 stg" CONFIGS="C3 C4 C5 C2" REPS=2 bash tools/ab.sh > gpurun_out/ab_stg.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
    tests/test_engine_e2e_gpu.py tests/test_kmer_gpu.py > gpurun_out/t_engine.log 2>&1 || { tail -20 gpurun_out/t_engine.log; exit 1; }
PAIRS=300000 timeout -k 10 300 python -u tools/detect_timing.py > gpurun_out/detect_timing.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/e2e_bench.py --pairs 10000000 --no-ref > gpurun_out/e2e_10M.txt 2>&1 || exit 1
echo ok
