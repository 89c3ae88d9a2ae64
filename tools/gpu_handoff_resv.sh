set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
for ev in 0 1000 100; do
  for n in K L; do
    EXOTIC_EVERY=$ev TAG="every=$ev $n" CONFIGS="C3 C5 C4" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
  done
done > gpurun_out/exotic3.txt
cat gpurun_out/exotic3.txt
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_engine_e2e_gpu.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pt_L.log 2>&1
rc=$?; tail -3 gpurun_out/pt_L.log; exit $rc
