set -u
PMC_GROUPS="sq" bash tools/pmc.sh && python tools/pmc_summary.py gpurun_out > gpurun_out/pmc_sum.txt || exit 1
touch fqtool_amd/csrc/pe_fast.hip && make STAMPS=1 engine > /dev/null 2>&1 || exit 1
VARIANTS=full timeout -k 10 300 python -u tools/ablate.py > gpurun_out/ablate_stamps.log 2>&1
rc=$?
touch fqtool_amd/csrc/pe_fast.hip && make engine > /dev/null 2>&1
exit $rc
