cd $GRAFT_REPO_ROOT
ALTS="E F" CONFIGS="C3 C5" REPS=2 bash tools/ab.sh > gpurun_out/ab4.txt 2>&1 || exit 1
CONFIG=C5 VARIANTS=full,no_trim,no_polyx,no_stats,no_overlap,no_filter,stage_only timeout -k 10 200 python tools/valu_probe.py > gpurun_out/c5_abl.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_engine2.log 2>&1
