set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for L in 250 150; do
 for mode in fast general; do
  if [ $mode = general ]; then export FQ_ENGINE_GENERAL_ONLY=1; else unset FQ_ENGINE_GENERAL_ONLY; fi
  timeout -k 10 300 python bench.py --config C3 --read-len $L --pairs 20000000 --steps 3 --warmup 1 --no-cpu-baseline --engine-pairs 0 --sample-pairs 200000 > gpurun_out/long_${L}_$mode.log 2>&1 || { tail -5 gpurun_out/long_${L}_$mode.log; exit 1; }
  grep '"metric"' gpurun_out/long_${L}_$mode.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L $mode', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'], d['parity_sample']['ok'])"
 done
done
