#!/bin/bash
# kernel + memory-copy trace of the fqtool binary on PAIRS synthetic pairs (raw stream)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
export FQ_TIMING=1  # (the binary otherwise ends with _exit, before the profiler writes its files)
D=$(mktemp -d /tmp/fqtrace_XXXX)
timeout -k 10 300 python -c "
import sys; sys.path.insert(0, 'tools'); sys.path.insert(0, '.')
import e2e_bench
print(e2e_bench.gen_fastq(${PAIRS:-10000000}, '$D'))
" > gpurun_out/trace_gen.log 2>&1 || { tail -5 gpurun_out/trace_gen.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/e2e_trace -o fq -- \
  ./fqtool_amd/bin/fqtool -i $D/r1.fq -I $D/r2.fq -o /dev/null -O /dev/null -q -a --detect_pe_adapter -g -w 16 \
  -J $D/r.json -H $D/r.html ${EXTRA:-} > gpurun_out/trace_run.log 2>&1 || { tail -5 gpurun_out/trace_run.log; exit 1; }
tail -3 gpurun_out/trace_run.log
rm -rf $D
find gpurun_out/e2e_trace -name "*.csv" | head
