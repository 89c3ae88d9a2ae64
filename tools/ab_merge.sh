# A/B: merge variant with quality rows in L2 (default build) vs staged in LDS (build/alt)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=full,no_stats,no_filter,no_polyg,stage_only
CONFIG=C4 VARIANTS=$V timeout -k 10 200 python tools/valu_probe.py > gpurun_out/ab_l2.txt 2>&1 || exit 1
CONFIG=C4 VARIANTS=$V FQ_ENGINE_LIB=$PWD/build/alt/libfqengine_qlds.so timeout -k 10 200 python tools/valu_probe.py > gpurun_out/ab_lds.txt 2>&1 || exit 1
paste gpurun_out/ab_l2.txt gpurun_out/ab_lds.txt
