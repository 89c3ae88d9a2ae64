#!/bin/bash
# PMC passes for the bench kernels (one counter group per rocprofv3 run; no trace domains mixed
# with --pmc).  Output: gpurun_out/pmc_<name>/..._counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd gpurun_out && export TMPDIR=/tmp && cd ..
ARGS="${PMC_BENCH_ARGS:---pairs 20000000 --steps 2 --warmup 1 --no-cpu-baseline}"
pass() {
    local name=$1; shift
    echo "== pmc $name: $*"
    timeout -k 10 600 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/pmc_$name -o pmc \
        -- python bench.py $ARGS > gpurun_out/pmc_$name.log 2>&1
    local rc=$?
    echo "pmc $name rc=$rc"
    return $rc
}
if [ "${PMC_LIST:-0}" = 1 ]; then
    timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
fi
for g in ${PMC_GROUPS:-fetch write sq lds}; do
    case $g in
    fetch) pass fetch FETCH_SIZE || exit $? ;;
    write) pass write WRITE_SIZE || exit $? ;;
    sq) pass sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY || exit $? ;;
    lds) pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $? ;;
    lds2) pass lds2 SQ_LDS_IDX_ACTIVE SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_VALU || exit $? ;;
    mem) pass mem SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY || exit $? ;;
    *) echo "unknown group $g"; exit 2 ;;
    esac
done
