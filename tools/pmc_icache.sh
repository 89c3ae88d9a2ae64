# profiling aid: instruction-cache counters of the bench kernels (one rocprofv3 --pmc pass each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
ARGS="--pairs 20000000 --steps 2 --warmup 1 --no-cpu-baseline"
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" "SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    name=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    echo "== $set"
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc_$name -o pmc -- python bench.py $ARGS > gpurun_out/pmc_$name.log 2>&1 || { echo "pass $name failed"; tail -5 gpurun_out/pmc_$name.log; }
done
python tools/pmc_summary.py gpurun_out > gpurun_out/pmc_sum.txt
