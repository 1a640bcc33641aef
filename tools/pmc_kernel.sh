#!/bin/bash
# Counter passes (one pass per group; no tracing domains besides kernel-trace)
# over tools/stage_bench.py for the kernels matching $1.
# usage: tools/pmc_kernel.sh <regex> <tag> [stage_bench args]
set -o pipefail
RE=$1; TAG=$2; shift 2
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -T --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- \
    python3 tools/stage_bench.py --reps 1 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
