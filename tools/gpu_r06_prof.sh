#!/bin/bash
# one GPU call (round 6): per config, the 100 M-pair kernel trace + HBM traffic passes
# (profile_round.sh) and the SQ issue / LDS passes (pmc_sq.sh), on the current build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
for c in ${CONFIGS:-C2 C5}; do
  ROUND=r06 CONFIG=$c bash tools/profile_round.sh > gpurun_out/profile_round_$c.log 2>&1 || { tail -5 gpurun_out/profile_round_$c.log; exit 1; }
  CONFIGS=$c KT=0 bash tools/pmc_sq.sh > gpurun_out/pmc_sq_$c.log 2>&1 || { tail -5 gpurun_out/pmc_sq_$c.log; exit 1; }
done
echo prof done
