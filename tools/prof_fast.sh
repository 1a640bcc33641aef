#!/bin/bash
# Kernel trace + counter passes for the fast pyramid kernel (one pass per group).
set -o pipefail
mkdir -p gpurun_out/pf
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf/trace -o run --output-format csv -- \
  python3 tools/stage_bench.py --fast --reps 2 > gpurun_out/pf/trace.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "pyr_fast" -d gpurun_out/pf/p$i -o run --output-format csv -- \
    python3 tools/stage_bench.py --fast --reps 1 > gpurun_out/pf/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
