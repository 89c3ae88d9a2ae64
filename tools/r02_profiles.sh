#!/bin/bash
# Round-2 profile set (GPU box): kernel trace + PMC HBM traffic of C4 and C5 at 100 M pairs,
# dynamic VALU/SALU/LDS instruction counts per tile of C3, C4, C5.  Every step has its own limit;
# the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${PROF_CONFIGS:-C4 C5}; do
    ROUND=r02 CONFIG=$c PAIRS=100000000 bash tools/profile_round.sh > gpurun_out/prof_$c.out 2>&1 || { echo "profile $c failed"; tail -5 gpurun_out/prof_$c.out; exit 1; }
    echo "profile $c ok"
done
for c in ${VALU_CONFIGS:-C3 C4 C5}; do
    CONFIG=$c bash tools/valu_probe.sh > gpurun_out/valu_$c.txt 2>&1 || { echo "valu $c failed"; exit 1; }
    echo "valu $c"; cat gpurun_out/valu_$c.txt
done
