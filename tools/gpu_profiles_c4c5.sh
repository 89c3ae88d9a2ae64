#!/bin/bash
# Round-3 kernel traces + PMC traffic of C4 and C5 (profile_round.sh) on the final build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in C4 C5; do
  ROUND=r03 CONFIG=$c bash tools/profile_round.sh > gpurun_out/profile_round_$c.log 2>&1 || { tail -5 gpurun_out/profile_round_$c.log; exit 1; }
  tail -2 gpurun_out/profile_round_$c.log
done
