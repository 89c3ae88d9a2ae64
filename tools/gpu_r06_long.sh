#!/bin/bash
# Round 6: the C3 kernel rate on 2x250 and 2x300 bp reads (the long320 build), 20 M pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
for L in 250 300; do
  timeout -k 10 300 python -u bench.py --read-len $L --pairs 20000000 --steps 5 --warmup 1 --no-cpu-baseline \
      --paths-pairs 0 --engine-pairs 0 > gpurun_out/r06_bench_c3_L$L.json 2> gpurun_out/r06_bench_c3_L$L.log || exit $?
done
