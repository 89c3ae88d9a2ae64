set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_engine_gpu.py tests/test_engine_e2e_gpu.py tests/test_fullsize_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_eng.log 2>&1; rc=$?; tail -3 gpurun_out/t_eng.log; [ $rc -eq 0 ] || exit $rc
for c in ${CFGS:-C4 C5 C3}; do timeout -k 10 300 python bench.py --config $c --pairs 100000000 --steps 5 --warmup 1 --no-cpu-baseline --engine-pairs 0 --sample-pairs 0 > gpurun_out/b_$c.log 2>&1 || exit $?; grep '"metric"' gpurun_out/b_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['roofline']['kernel_ms_avg'], d['roofline']['frac'])"; done
if [ -n "${VPROBE:-}" ]; then for c in $VPROBE; do CONFIG=$c VARIANTS=${VARIANTS:-full,no_polyg} timeout -k 10 200 python tools/valu_probe.py || exit 1; done; fi
