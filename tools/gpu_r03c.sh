#!/bin/bash
# round-3 GPU step: lowercase bases on the fast kernels (parity + cost), the paths leg, and the
# e2e tool (text packs vs tiles, one vs several engines)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_engine_gpu.py \
    -m gpu > gpurun_out/t_engine_low.log 2>&1 || { tail -30 gpurun_out/t_engine_low.log; exit 1; }
ALTS="head low" CONFIGS="C3 C4 C5" REPS=2 bash tools/ab.sh > gpurun_out/ab_lowercase.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_paths.json \
    2> gpurun_out/bench_paths.log || exit 1
timeout -k 10 600 python -u tools/e2e_bench.py --pairs 10000000 --no-ref --repeat 2 > gpurun_out/e2e_r03c.txt 2>&1 || exit 1
FQ_TEXT_MODE=0 timeout -k 10 300 python -u tools/e2e_bench.py --pairs 10000000 --no-ref >> gpurun_out/e2e_r03c.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/e2e_bench.py --pairs 10000000 --no-ref --devices 0,0 >> gpurun_out/e2e_r03c.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/e2e_bench.py --pairs 10000000 --no-ref --devices 0,0,0,0 >> gpurun_out/e2e_r03c.txt 2>&1 || exit 1
echo ok
