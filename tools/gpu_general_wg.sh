#!/bin/bash
# one GPU call: general kernel workgroup size A/B (P0: 256 threads, P1: 512) -- general-only C3,
# 1 % hand-off pairs, clean C3 -- then the engine / e2e / host GPU tests on the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for n in P0 P1; do
  FQ_ENGINE_GENERAL_ONLY=1 LAUNCHES=3 TAG="general $n" CONFIGS="C3" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 240 python tools/ab_time.py 2>&1 | grep median || exit 1
  EXOTIC_EVERY=100 TAG="every=100 $n" CONFIGS="C3 C5" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
  TAG="clean $n" CONFIGS="C3" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
done > gpurun_out/general_wg.txt
cat gpurun_out/general_wg.txt
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_engine_e2e_gpu.py tests/test_host_e2e.py tests/test_dup_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pt_wg.log 2>&1
rc=$?; tail -3 gpurun_out/pt_wg.log; exit $rc
