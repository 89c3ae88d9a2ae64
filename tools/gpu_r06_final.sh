#!/bin/bash
# Round 6 on the GPU box: smoke() and the default bench run (every leg), as the driver runs them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_smoke.log 2>&1 || exit $?
timeout -k 10 1000 python -u bench.py > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.log
