set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_engine_e2e_gpu.py -k "C4 or merge or PE_correct or umi" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_longmerge.log 2>&1; rc=$?; tail -3 gpurun_out/t_longmerge.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -k "PE_umi_merge" -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/t_umimerge_full.log 2>&1; rc=$?; tail -3 gpurun_out/t_umimerge_full.log; [ $rc -eq 0 ] || exit $rc
TAG=fast_L250 PAIRS=4000000 L=250 STRIDE=256 CONFIGS="C4 C3" timeout -k 10 300 python tools/ab_time.py || exit $?
TAG=fast_L300 PAIRS=4000000 L=300 STRIDE=304 CONFIGS="C4" timeout -k 10 300 python tools/ab_time.py || exit $?
TAG=general_L250 LAUNCHES=3 FQ_ENGINE_GENERAL_ONLY=1 PAIRS=4000000 L=250 STRIDE=256 CONFIGS="C4" timeout -k 10 300 python tools/ab_time.py || exit $?
TAG=umi8 UMI=8 CONFIGS="C4" timeout -k 10 300 python tools/ab_time.py || exit $?
