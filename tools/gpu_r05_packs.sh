#!/bin/bash
# one GPU call (round 5): e2e at 50 M pairs (outputs /dev/null) by raw pack size (page-locked
# stages scale with it; the exit releases them)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V="${VARIANTS:-;--pack_pairs 65536;--pack_pairs 98304;--pack_pairs 65536 FQ_RAW_STAGES=12}"
timeout -k 10 900 python -u tools/e2e_bench.py --pairs ${PAIRS:-50000000} --no-ref --null-out --pause 2 --repeat ${REPEAT:-3} \
   --variants "$V" > gpurun_out/e2e_packs.txt 2>&1 || exit 1
