# profiling aid: one bench line per BASELINE workload on this GPU (C2 SE, C3, C4 merge, C5 full)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in ${CONFIGS:-C2 C3 C4 C5}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --pairs ${PAIRS:-20000000} --config $c --steps 5 --warmup 1 > gpurun_out/cfg_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/cfg_$c.log; exit 1; }
  echo "$c $(grep '"metric"' gpurun_out/cfg_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms", "frac", d["roofline"]["frac"])')"
done
