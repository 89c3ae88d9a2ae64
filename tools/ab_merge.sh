# A/B of merge-variant layouts (profiling builds under build/alt): kernel ms per ablation variant
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=${VARIANTS:-full,no_stats,no_filter,stage_only}
CONFIG=${CONFIG:-C4} VARIANTS=$V timeout -k 10 200 python tools/valu_probe.py > gpurun_out/ab_A.txt 2>&1 || exit 1
for n in ${ALTS:-B C D}; do
  CONFIG=${CONFIG:-C4} VARIANTS=$V FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 200 python tools/valu_probe.py > gpurun_out/ab_$n.txt 2>&1 || exit 1
done
paste gpurun_out/ab_A.txt $(for n in ${ALTS:-B C D}; do echo gpurun_out/ab_$n.txt; done) | grep -v amdgpu.ids
