#!/bin/bash
# one GPU call: UMI / index filter on the fast kernels vs the previous build, clean configs,
# then the engine / full-size / e2e / host GPU tests on the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for n in ${UMI_ALTS:-G I}; do
  for v in "UMI=0" "UMI=8" "INDEX_EVERY=100"; do
    env $v TAG="$v $n" CONFIGS="${CONFIGS:-C3 C5}" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 240 python tools/ab_time.py 2>&1 | grep median || exit 1
  done
done > gpurun_out/umi_ab.txt
cat gpurun_out/umi_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_engine_e2e_gpu.py tests/test_host_e2e.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pt_umi.log 2>&1
rc=$?; tail -5 gpurun_out/pt_umi.log; exit $rc
