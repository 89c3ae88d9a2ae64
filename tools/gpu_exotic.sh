#!/bin/bash
# one GPU call: kernel ms with every k-th pair holding a lowercase base (hand-off to the general
# kernel), tile hand-off build (A) vs per-pair hand-off build (C); then the whole GPU suite + smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for ev in 0 1000 100; do
  for n in ${ALTS:-A C}; do
    EXOTIC_EVERY=$ev TAG="every=$ev $n" CONFIGS="${CONFIGS:-C3 C5}" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
  done
done > gpurun_out/exotic.txt
cat gpurun_out/exotic.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
