set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_engine_e2e_gpu.py tests/test_host_e2e.py -k "complexity or correct_front or umi_merge or correct_merge" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_cplx.log 2>&1; rc=$?; tail -3 gpurun_out/t_cplx.log; exit $rc
