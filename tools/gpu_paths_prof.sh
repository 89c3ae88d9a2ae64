#!/bin/bash
# one GPU call: rocprofv3 kernel traces of the non-default paths at 20 M pairs (general kernel
# only; -c and UMI on the fast kernels; 1 % hand-off pairs), each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
R=$PWD; export TMPDIR=/tmp
prof() {  # name, then env assignments are already exported by the caller
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$1 -o $1 -- python3 $R/tools/ab_time.py > $R/gpurun_out/prof_$1.log 2>&1 || exit 1
    grep median $R/gpurun_out/prof_$1.log
}
(export FQ_ENGINE_GENERAL_ONLY=1 CONFIGS=C3 LAUNCHES=3; prof general_c3) || exit 1
(export CORRECT=1 CONFIGS="C3 C5" LAUNCHES=4; prof correct) || exit 1
(export UMI=8 CONFIGS="C3 C5" LAUNCHES=4; prof umi) || exit 1
(export EXOTIC_EVERY=100 CONFIGS="C3" LAUNCHES=4; prof exotic) || exit 1
