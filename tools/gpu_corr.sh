set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_engine_e2e_gpu.py -k "correct or umi" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_corr.log 2>&1; rc=$?; tail -3 gpurun_out/t_corr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -k "PE_correct_front or PE_correct_umi_merge" -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/t_corr_full.log 2>&1; rc=$?; tail -3 gpurun_out/t_corr_full.log; [ $rc -eq 0 ] || exit $rc
TAG=correct_umi8 CORRECT=1 UMI=8 CONFIGS="C3 C4" timeout -k 10 300 python tools/ab_time.py || exit $?
