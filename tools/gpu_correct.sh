set -u
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out
for n in C E; do
  for c in 0 1; do
    CORRECT=$c TAG="correct=$c $n" CONFIGS="C3 C5" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
  done
done > gpurun_out/correct_ab.txt
cat gpurun_out/correct_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py tests/test_engine_e2e_gpu.py tests/test_host_e2e.py -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pt_correct.log 2>&1
rc=$?; tail -5 gpurun_out/pt_correct.log; exit $rc
