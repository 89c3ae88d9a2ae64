#!/bin/bash
# round-3 GPU step: text-pack parity, tool byte-identity on the golden cases, e2e timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_text_gpu.py \
    tests/test_host_e2e.py -m gpu > gpurun_out/t_text.log 2>&1 || { tail -30 gpurun_out/t_text.log; exit 1; }
timeout -k 10 600 python -u tools/e2e_bench.py --pairs 10000000 --no-ref > gpurun_out/e2e_text_10M.txt 2>&1 || exit 1
FQ_TEXT_MODE=0 timeout -k 10 600 python -u tools/e2e_bench.py --pairs 10000000 --no-ref > gpurun_out/e2e_tiles_10M.txt 2>&1 || exit 1
ALTS="m16 m12 m8" CONFIGS="C4" REPS=2 bash tools/ab.sh > gpurun_out/ab_merge_waves.txt 2>&1 || exit 1
echo ok
