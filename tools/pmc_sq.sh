#!/bin/bash
# SQ / GRBM counter passes (issue, waits, LDS) of the fast kernel on the bench workloads, one
# rocprofv3 --pmc run per (config, group), kernel trace in its own run.  Run on the GPU box:
#   ROUND=r03 CONFIGS="C3 C4 C5" bash tools/pmc_sq.sh
# Output: gpurun_out/sq/<cfg>_<group>/..._counter_collection.csv, gpurun_out/sq/<cfg>_kt/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PAIRS=${PAIRS:-100000000}
OUT=gpurun_out/sq
mkdir -p $OUT
for cfg in ${CONFIGS:-C3 C4 C5}; do
  ARGS="--config $cfg --pairs $PAIRS --steps 2 --warmup 1 --no-cpu-baseline --sample-pairs 0 --engine-pairs 0 --paths-pairs 0"
  if [ "${KT:-1}" = 1 ]; then
    echo "== $cfg kernel trace"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${cfg}_kt -o kt -- \
        python3 bench.py $ARGS > $OUT/${cfg}_kt.log 2>&1 || { echo "kt $cfg failed rc=$?"; exit 1; }
  fi
  for g in ${GROUPS_SQ:-issue lds}; do
    case $g in
    issue) C="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" ;;
    lds) C="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE" ;;
    *) echo "unknown group $g"; exit 2 ;;
    esac
    echo "== $cfg pmc $g"
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $OUT/${cfg}_$g -o pmc -- \
        python3 bench.py $ARGS > $OUT/${cfg}_$g.log 2>&1 || { echo "pmc $cfg $g failed rc=$?"; exit 1; }
  done
done
echo "pmc_sq done"
