set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py -k "adapter_by_sequence or C3b or SE_adapter or PE_merge_q or PE_correct or PE_all" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_adseq.log 2>&1; rc=$?; tail -3 gpurun_out/t_adseq.log; [ $rc -eq 0 ] || exit $rc
TAG=adseq ADAPTERS=1 CONFIGS="C3 C5" timeout -k 10 300 python tools/ab_time.py || exit $?
TAG=plain CONFIGS="C3 C4" timeout -k 10 300 python tools/ab_time.py || exit $?
TAG=correct CORRECT=1 CONFIGS="C3 C4" timeout -k 10 300 python tools/ab_time.py || exit $?
timeout -k 10 600 python -u -m pytest tests/test_fullsize_gpu.py -k "C3b or PE_correct_merge" -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/t_adseq_full.log 2>&1; rc=$?; tail -3 gpurun_out/t_adseq_full.log; exit $rc
