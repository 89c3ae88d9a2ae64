set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_host_e2e.py tests/test_engine_e2e_gpu.py -k "raw or td_pe_qag or synth or binary" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_stages.log 2>&1; rc=$?; tail -2 gpurun_out/t_stages.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/e2e_bench.py --pairs 50000000 --no-ref --null-out --repeat 2 --variants "FQ_RAW_STAGES=9;FQ_RAW_STAGES=13;FQ_RAW_STAGES=17" > gpurun_out/e2e_stages.txt 2>&1 || exit 1
grep -h Mreads_s gpurun_out/e2e_stages.txt | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['extra'], d['Mreads_s'], d['wall_s'], d['tool_log'][120:420])"
