#!/bin/bash
# one GPU call (round 5): kernel + copy traces of the fqtool binary, C3 and C4 (-m) options, 20 M pairs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
PAIRS=${PAIRS:-20000000} bash tools/gpu_e2e_trace.sh > gpurun_out/e2e_trace_c3.log 2>&1 || exit 1
mv gpurun_out/e2e_trace gpurun_out/e2e_trace_c3
PAIRS=${PAIRS:-20000000} EXTRA="--enable_cut_right -m --merge_output /dev/null" bash tools/gpu_e2e_trace.sh > gpurun_out/e2e_trace_c4.log 2>&1 || exit 1
mv gpurun_out/e2e_trace gpurun_out/e2e_trace_c4
