set -u
for m in "OPAQUE_NCH=0" "OPAQUE_NCH=0 SCHED_PIN=0" "OPAQUE_NCH=1"; do
  touch fqtool_amd/csrc/pe_fast.hip
  make $m engine > /dev/null 2>&1 || { echo "build failed"; exit 1; }
  for c in C3 C2 C5; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --pairs 20000000 --config $c > gpurun_out/p_$c.log 2>&1 || exit 1
    echo "$m $c $(tail -n 1 gpurun_out/p_$c.log | cut -c1-100)"
  done
done
touch fqtool_amd/csrc/pe_fast.hip
