set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_long.log 2>&1; rc=$?; tail -15 gpurun_out/t_long.log; [ $rc -eq 0 ] || exit $rc
for L in 250 300 150; do
  timeout -k 10 300 python bench.py --config C3 --read-len $L --pairs 20000000 --steps 3 --warmup 1 --no-cpu-baseline --engine-pairs 0 --sample-pairs 200000 > gpurun_out/long_${L}.log 2>&1 || { tail -5 gpurun_out/long_${L}.log; exit 1; }
  grep '"metric"' gpurun_out/long_${L}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'], d['parity_sample']['ok'])"
done
