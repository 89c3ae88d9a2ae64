set -u; cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_host_e2e.py tests/test_kmer_gpu.py tests/test_dup_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_host.log 2>&1; rc=$?; tail -3 gpurun_out/t_host.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config C3 --steps 3 --warmup 1 --engine-pairs 0 --sample-pairs 0 > gpurun_out/b_e2e.log 2>&1 || { tail -5 gpurun_out/b_e2e.log; exit 1; }
grep '"metric"' gpurun_out/b_e2e.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('e2e'))"
