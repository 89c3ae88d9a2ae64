#!/bin/bash
# Profiling aid: kernel ms of engine variants (build/alt/lib_<name>.so, tools/ab_build.sh) per config,
# alternating the variants REPS times.  ALTS="A B C" CONFIGS="C3 C5" REPS=2 bash tools/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
  for n in ${ALTS:-A B}; do
    TAG="rep$rep $n" CONFIGS="${CONFIGS:-C3}" FQ_ENGINE_LIB=$PWD/build/alt/lib_$n.so timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
  done
done
