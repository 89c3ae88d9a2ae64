#!/bin/bash
# Round profile of one bench workload (run on the GPU box; gpurun brings gpurun_out/ back, then
# copy gpurun_out/round_profiles/* into profiles/):
#   rocprofv3 --kernel-trace --stats  -> <round>_kernel_stats_<config>.csv (+ the bench line)
#   PMC FETCH_SIZE / WRITE_SIZE passes -> <round>_pmc_<config>.json (bench.py's roofline.traffic)
set -u
ROUND=${ROUND:-r01}
CFG=${CONFIG:-C3}
PAIRS=${PAIRS:-100000000}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/round_profiles
OUT=gpurun_out/round_profiles
export TMPDIR=/tmp
ARGS="--config $CFG --pairs $PAIRS --steps 5 --warmup 1 --no-cpu-baseline --paths-pairs 0"
rm -rf gpurun_out/kt_$CFG gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$CFG -o kt -- python3 bench.py $ARGS \
    > gpurun_out/kt_$CFG.log 2>&1 || { echo "kernel trace failed rc=$?"; exit 1; }
stats=$(find gpurun_out/kt_$CFG -name '*kernel_stats.csv' | head -n 1)
[ -n "$stats" ] || { echo "no kernel_stats.csv"; exit 1; }
cp "$stats" $OUT/${ROUND}_kernel_stats_$CFG.csv
grep '"metric"' gpurun_out/kt_$CFG.log | tail -n 1 > $OUT/${ROUND}_kernel_stats_${CFG}_bench.json
PMC_BENCH_ARGS="$ARGS" PMC_GROUPS="fetch write" bash tools/pmc.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out --config $CFG --pairs $PAIRS > $OUT/${ROUND}_pmc_$CFG.json || exit 1
cat $OUT/${ROUND}_kernel_stats_$CFG.csv $OUT/${ROUND}_pmc_$CFG.json
