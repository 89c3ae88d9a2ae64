# profiling aid: SQ counters of the stage-only fast kernel (ABLATE_STAGE=1) and of stagebench
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
touch fqtool_amd/csrc/pe_fast.hip
make ABLATE_STAGE=1 engine > /dev/null 2>&1 || { echo "build failed"; exit 1; }
rm -rf gpurun_out/spmc_*
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
VARIANTS=stage_only timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/spmc_k -o pmc -- python3 tools/ablate.py > gpurun_out/spmc_k.log 2>&1 || { echo "k failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/spmc_m -o pmc -- tools/micro/stagebench > gpurun_out/spmc_m.log 2>&1 || { echo "m failed"; exit 1; }
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM"
VARIANTS=stage_only timeout -k 10 300 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/spmc_k2 -o pmc -- python3 tools/ablate.py > gpurun_out/spmc_k2.log 2>&1 || { echo "k2 failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/spmc_m2 -o pmc -- tools/micro/stagebench > gpurun_out/spmc_m2.log 2>&1 || { echo "m2 failed"; exit 1; }
touch fqtool_amd/csrc/pe_fast.hip
echo done
