#!/bin/bash
# SQ / LDS counter passes of the fast kernel for several bench workloads (one rocprofv3 run per
# counter group and config; no trace domains mixed with --pmc).  Summary: tools/pmc_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in ${CONFIGS:-C3 C4 C5}; do
    for g in ${PMC_SETS:-sq lds2}; do
        case $g in
        sq) C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" ;;
        lds2) C="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU" ;;
        *) echo "unknown group $g"; exit 2 ;;
        esac
        echo "== $cfg $g"
        timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${cfg}_$g -o pmc \
            -- python3 bench.py --config $cfg --pairs ${PAIRS:-20000000} --steps 2 --warmup 1 --no-cpu-baseline \
               --sample-pairs 0 --engine-pairs 0 > gpurun_out/pmc_${cfg}_$g.log 2>&1 || { echo "rc=$?"; exit 1; }
    done
done
python3 tools/pmc_summary.py gpurun_out
