#!/bin/bash
# Round 6: VALU / LDS instructions of the fast kernel with phases switched off (tools/ablate.py's
# fq_params.reserved[0] bits), one rocprofv3 --pmc run: launches come in variant order (3 reps x
# 2 launches x variants, then the stamped run).  Parsed by hand from gpurun_out/vs/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/vs
VARIANTS=${VARIANTS:-full,no_overlap,no_filter,no_stats,no_polyg,stage_only} CONFIG=${CONFIG:-C3} \
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS --output-format csv -d gpurun_out/vs -o pmc -- \
  python3 tools/ablate.py > gpurun_out/vs/log.txt 2>&1
