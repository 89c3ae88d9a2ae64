#!/bin/bash
# Profiling aid: median kernel ms of the fast kernel with phases switched off (pe_fast.hip ablation
# bits), per config.  CONFIGS="C4 C5" bash tools/ablate_cfg.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in full:0 no_overlap:1 no_filter:2 no_stats:4 no_polyg:8 no_trim:1024 no_polyx:2048 stage_only:15; do
  ABL=${v#*:} TAG=${v%%:*} CONFIGS="${CONFIGS:-C3}" timeout -k 10 180 python tools/ab_time.py 2>&1 | grep median || exit 1
done
