# profiling aid: fast-kernel time vs the staging look-ahead (make AHEAD=n)
set -u
for a in ${AHEADS:-3 5 7 10}; do
  touch fqtool_amd/csrc/pe_fast.hip
  make AHEAD=$a engine > /dev/null 2>&1 || { echo "build $a failed"; exit 1; }
  echo "== AHEAD=$a"
  VARIANTS=full,stage_only timeout -k 10 200 python tools/ablate.py > gpurun_out/ahead$a.log 2>&1 || { echo "ablate $a failed"; exit 1; }
  grep -E "full|stage_only" gpurun_out/ahead$a.log
done
touch fqtool_amd/csrc/pe_fast.hip
make engine > /dev/null 2>&1
