# profiling aid: stage-only time vs batch size (fixed per-launch cost vs per-tile cost)
set -u
touch fqtool_amd/csrc/pe_fast.hip
make ABLATE_STAGE=1 engine > /dev/null 2>&1 || { echo "build failed"; exit 1; }
for n in 200000 2000000 20000000; do
  PAIRS=$n timeout -k 10 200 python tools/ablate.py > gpurun_out/sf$n.log 2>&1 || { echo "ablate $n failed"; exit 1; }
  echo "pairs $n: $(grep -E 'stage_only' gpurun_out/sf$n.log)"
done
touch fqtool_amd/csrc/pe_fast.hip
