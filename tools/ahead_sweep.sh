set -u
for a in 3 5 7; do
  touch fqtool_amd/csrc/pe_fast.hip
  make AHEAD=$a engine > /dev/null 2>&1 || { echo "build $a failed"; exit 1; }
  timeout -k 10 200 python bench.py --no-cpu-baseline --pairs 20000000 --config C3 > gpurun_out/ah$a.log 2>&1 || { echo "bench $a failed"; exit 1; }
  echo "ahead $a: $(tail -n 1 gpurun_out/ah$a.log | cut -c1-120)"
done
