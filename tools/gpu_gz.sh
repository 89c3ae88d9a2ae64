set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_host_e2e.py -k "gz or bgzf or td_pe_qag or td_se_q" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_gz.log 2>&1; rc=$?; tail -2 gpurun_out/t_gz.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/e2e_bench.py --pairs 10000000 --no-ref --null-out --gz bgzf --repeat 2 > gpurun_out/e2e_gz.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/e2e_bench.py --pairs 2000000 --no-ref --null-out --gz gzip >> gpurun_out/e2e_gz.txt 2>&1 || exit 1
grep -h Mreads_s gpurun_out/e2e_gz.txt | python -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['pairs'], d['Mreads_s'], d['wall_s'], d['tool_log'][:300])"
