#!/bin/bash
# Round profile of one bench workload, copied into profiles/ (run on the GPU box):
#   rocprofv3 --kernel-trace --stats  -> profiles/<round>_kernel_stats_<config>.csv
#   PMC FETCH_SIZE / WRITE_SIZE passes -> profiles/<round>_pmc_<config>.json (bench.py's roofline.traffic)
set -u
ROUND=${ROUND:-r01}
CFG=${CONFIG:-C3}
PAIRS=${PAIRS:-100000000}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
ARGS="--config $CFG --pairs $PAIRS --steps 5 --warmup 1 --no-cpu-baseline"
rm -rf gpurun_out/kt_$CFG gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$CFG -o kt -- python3 bench.py $ARGS \
    > gpurun_out/kt_$CFG.log 2>&1 || { echo "kernel trace failed rc=$?"; exit 1; }
stats=$(find gpurun_out/kt_$CFG -name '*kernel_stats.csv' | head -n 1)
[ -n "$stats" ] || { echo "no kernel_stats.csv"; exit 1; }
cp "$stats" profiles/${ROUND}_kernel_stats_$CFG.csv
tail -n 1 gpurun_out/kt_$CFG.log > profiles/${ROUND}_kernel_stats_${CFG}_bench.json
PMC_BENCH_ARGS="$ARGS" PMC_GROUPS="fetch write" bash tools/pmc.sh || exit 1
python3 tools/pmc_traffic.py gpurun_out --config $CFG --pairs $PAIRS > profiles/${ROUND}_pmc_$CFG.json || exit 1
cat profiles/${ROUND}_kernel_stats_$CFG.csv profiles/${ROUND}_pmc_$CFG.json
