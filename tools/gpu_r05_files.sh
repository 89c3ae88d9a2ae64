#!/bin/bash
# one GPU call (round 5): e2e with plain FASTQ output files at 50 M pairs (positional writes on
# I/O threads), GPU text egress and records-only egress as byte ranges
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 900 python -u tools/e2e_bench.py --pairs ${PAIRS:-50000000} --no-ref --pause 2 --repeat ${REPEAT:-2} \
   --variants "${VARIANTS:-;FQ_RAW_EGRESS=host}" > gpurun_out/e2e_files.txt 2>&1 || exit 1
