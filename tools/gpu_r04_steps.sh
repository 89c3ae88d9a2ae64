#!/bin/bash
# Round-4 GPU call: the steps named in STEPS, in order, each under its own time limit; stops at the
# first failure.  Outputs under gpurun_out/.
#   STEPS="ab tests prof:C3 prof:C4 e2e_gz bench sq:C3"  ALTS=..  CONFIGS=..  TESTS=..
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for st in ${STEPS:-}; do
  echo "== step $st $(date +%T)"
  case $st in
  opcost) timeout -k 10 200 ./build/micro/opcost2 > gpurun_out/opcost2.txt 2>&1 || exit 1 ;;
  sel) timeout -k 10 200 ./build/micro/sel > gpurun_out/sel.txt 2>&1 || exit 1 ;;
  ab) ALTS="${ALTS:-base}" CONFIGS="${CONFIGS:-C3}" REPS=${REPS:-2} bash tools/ab.sh > gpurun_out/ab.txt 2>&1 || exit 1 ;;
  tests) timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_engine_gpu.py tests/test_fullsize_gpu.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/pt.log 2>&1 || exit 1 ;;
  htests) timeout -k 10 900 python -u -m pytest tests/test_host_e2e.py -m gpu -k "${HTESTS:-raw_stream}" -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_host.log 2>&1 || exit 1 ;;
  prof:*) c=${st#prof:}
    CONFIG=$c PAIRS=20000000 bash tools/valu_probe.sh > gpurun_out/vprobe_sum_$c.txt 2>&1 || exit 1
    CONFIG=$c VARIANTS=full FQ_ENGINE_LIB=$PWD/build/alt/lib_stamps.so timeout -k 10 300 python -u tools/ablate.py > gpurun_out/stamps_$c.txt 2>&1 || exit 1 ;;
  e2e_gz) timeout -k 10 400 python -u tools/e2e_bench.py --pairs ${GZ_PAIRS:-4000000} --gz gzip --no-ref --null-out --repeat 2 > gpurun_out/e2e_gz.txt 2>&1 || exit 1 ;;
  e2e:*) d=${st#e2e:}; timeout -k 10 500 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-20000000} --no-ref --null-out --repeat 3 --devices $d ${E2E_ARGS:-} > gpurun_out/e2e_$d.txt 2>&1 || exit 1 ;;
  e2e_multi) timeout -k 10 600 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-20000000} --no-ref --null-out --repeat 3 --variants "--devices 0;--devices 0,0;--devices 0,0,0" > gpurun_out/e2e_multi.txt 2>&1 || exit 1 ;;
  e2e_pause) timeout -k 10 500 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-20000000} --no-ref --null-out --repeat 3 --pause ${E2E_PAUSE:-2} > gpurun_out/e2e_pause.txt 2>&1 || exit 1 ;;
  e2e_numa) timeout -k 10 700 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-50000000} --no-ref --null-out --repeat 3 --pause 2 --variants "FQ_NUMA=0;FQ_NUMA=1" > gpurun_out/e2e_numa.txt 2>&1 || exit 1 ;;
  e2e_var) timeout -k 10 900 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-50000000} --no-ref --null-out --repeat ${E2E_REPEAT:-3} --pause 2 --variants "${E2E_VARIANTS}" > gpurun_out/e2e_var.txt 2>&1 || exit 1 ;;
  e2e_noegress) FQ_PROF_NO_EGRESS=1 timeout -k 10 500 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-20000000} --no-ref --null-out --repeat 3 > gpurun_out/e2e_noegress.txt 2>&1 || exit 1 ;;
  e2e_hostegress) FQ_RAW_EGRESS=host timeout -k 10 500 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-20000000} --no-ref --null-out --repeat 3 > gpurun_out/e2e_hostegress.txt 2>&1 || exit 1 ;;
  htests_hostegress) FQ_RAW_EGRESS=host timeout -k 10 900 python -u -m pytest tests/test_host_e2e.py -m gpu -k "${HTESTS:-raw_stream}" -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_host_hostegress.log 2>&1 || exit 1 ;;
  e2e_early) FQ_DETECT_EARLY=1 timeout -k 10 500 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-20000000} --no-ref --null-out --repeat 3 > gpurun_out/e2e_early.txt 2>&1 || exit 1 ;;
  e2e) timeout -k 10 500 python -u tools/e2e_bench.py --pairs ${E2E_PAIRS:-20000000} --no-ref --null-out --repeat 3 ${E2E_ARGS:-} > gpurun_out/e2e.txt 2>&1 || exit 1 ;;
  bench) timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.log || exit 1 ;;
  round:*) c=${st#round:}; ROUND=r04 CONFIG=$c timeout -k 10 1000 bash tools/profile_round.sh > gpurun_out/profile_round_$c.log 2>&1 || exit 1 ;;
  sq:*) c=${st#sq:}; ROUND=r04 CONFIGS=$c timeout -k 10 900 bash tools/pmc_sq.sh > gpurun_out/pmc_sq_$c.log 2>&1 || exit 1 ;;
  *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo "== steps done $(date +%T)"
