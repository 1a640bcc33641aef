#!/bin/bash
# Counter passes over the SIFT_FLAG_FAST pyramid (pyr_tri_kernel), one
# rocprofv3 process per group, kernel-trace only beside the counters.
# usage: tools/pmc_tri.sh <tag>
set -o pipefail
TAG=${1:-tri}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM" \
           "SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INST_LEVEL_VMEM SQ_LDS_UNALIGNED_STALL" \
           "TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum" ; do
  i=$((i+1))
  timeout -k 5 -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -T --kernel-include-regex "pyr_tri" -d $OUT/p$i -o run --output-format csv -- \
    python3 tools/stage_bench.py --reps 1 --fast > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT > $OUT/table.txt && cat $OUT/table.txt
