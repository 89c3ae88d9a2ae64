#!/bin/bash
# Round 6 on the GPU box: the parallel inflater's speed probe (tools/pargz_speed.py), then bench.py
# with its host legs at 10M pairs (e2e on plain and on single-member gzip -6 inputs, the reference
# on both).  FILE_LEGS=1 adds the file-output legs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
[ "${SPEED:-1}" = 0 ] || timeout -k 10 400 python -u tools/pargz_speed.py --reads "${READS:-6000000}" --threads 1,4,8,16 \
    --out gpurun_out/r06_pargz_speed.json > gpurun_out/r06_pargz_speed.log 2>&1 || exit $?
FQ_BENCH_FILE_LEGS=${FILE_LEGS:-0} timeout -k 10 900 python -u bench.py --steps 3 --warmup 1 \
    --e2e-pairs "${E2E_PAIRS:-10000000}" > gpurun_out/r06_bench_gzin.json 2> gpurun_out/r06_bench_gzin.log
