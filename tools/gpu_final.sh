#!/bin/bash
# one GPU call: hand-off rate of the previous build (I) vs the current one (J) on inputs with
# lowercase bases, then the full refresh (tests, smoke, profiles, config lines, bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for ev in 0 1000 100; do
  for n in ${ALTS:-I J}; do
    EXOTIC_EVERY=$ev TAG="every=$ev $n" CONFIGS="C3 C5" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
  done
done > gpurun_out/exotic2.txt
cat gpurun_out/exotic2.txt
bash tools/gpu_refresh.sh
