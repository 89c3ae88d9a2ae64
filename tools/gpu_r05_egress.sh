#!/bin/bash
# one GPU call (round 5): the raw stream's egress modes at 50 M pairs, outputs to /dev/null, then to
# plain files at 20 M pairs (GPU output text / records-only with byte ranges / records-only copied)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
V=";FQ_RAW_EGRESS=host;FQ_RAW_EGRESS=host FQ_RAW_ZC=0"
timeout -k 10 700 python -u tools/e2e_bench.py --pairs ${PAIRS:-50000000} --no-ref --null-out --pause 2 --repeat ${REPEAT:-3} \
   --variants "$V" > gpurun_out/e2e_egress_zc.txt 2>&1 || exit 1
timeout -k 10 500 python -u tools/e2e_bench.py --pairs ${FPAIRS:-20000000} --no-ref --pause 2 --repeat 2 \
   --variants "$V" > gpurun_out/e2e_egress_zc_file.txt 2>&1 || exit 1
