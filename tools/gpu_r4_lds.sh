#!/bin/bash
# LDS-array occupancy: SQ_LDS_IDX_ACTIVE and friends for the exact kernels and pyr_tri_kernel (one PMC group, own runs)
set -o pipefail
OUT=gpurun_out/prof_lds
mkdir -p $OUT
export TMPDIR=/tmp
G="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $G -T --kernel-include-regex "descriptor_kernel|blur_sym_kernel|orient_slots_kernel|extrema_walk_kernel" \
  -d $OUT/x -o run --output-format csv -- python3 tools/stage_bench.py --reps 1 > $OUT/x.log 2>&1 || { tail -5 $OUT/x.log; exit 1; }
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $G -T --kernel-include-regex "pyr_tri" \
  -d $OUT/f -o run --output-format csv -- python3 tools/stage_bench.py --reps 1 --fast > $OUT/f.log 2>&1 || { tail -5 $OUT/f.log; exit 1; }
echo lds done
