# profiling aid: stage-only time with the staging work ablated (make ABLATE_STAGE=n)
set -u
for a in 0 1 2; do
  touch fqtool_amd/csrc/pe_fast.hip
  make ABLATE_STAGE=$a engine > /dev/null 2>&1 || { echo "build $a failed"; exit 1; }
  echo "== ABLATE_STAGE=$a"
  timeout -k 10 200 python tools/ablate.py > gpurun_out/stage$a.log 2>&1 || { echo "ablate $a failed"; exit 1; }
  grep -E "full|stage_only|no_overlap_filter_stats" gpurun_out/stage$a.log
done
touch fqtool_amd/csrc/pe_fast.hip
