#!/bin/bash
# one GPU call (round 4): per-phase dynamic VALU counts (valu_probe, ablation variants under
# rocprofv3 --pmc) for CONFIGS, and per-phase wave cycles from the stamps build (lib_stamps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CONFIGS:-C3}; do
  CONFIG=$c PAIRS=20000000 bash tools/valu_probe.sh > gpurun_out/vprobe_sum_$c.txt 2>&1 || exit 1
  CONFIG=$c VARIANTS=full FQ_ENGINE_LIB=$PWD/build/alt/lib_stamps.so timeout -k 10 300 python -u tools/ablate.py > gpurun_out/stamps_$c.txt 2>&1 || exit 1
done
exit 0
