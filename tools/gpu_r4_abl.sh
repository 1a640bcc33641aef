#!/bin/bash
# GPU call: tri ablations (store / DMA contributions) + memory-pipe counters.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=3 bash tools/ab_var.sh r4abl prod abl1 abl2 abl3 abl4 || exit 1
OUT=gpurun_out/pmc_tri4b
mkdir -p $OUT
i=0
for grp in "TA_BUFFER_READ_LDS_WAVEFRONTS_sum TA_BUFFER_WRITE_WAVEFRONTS_sum TD_STORE_WAVEFRONT_sum TD_LOAD_WAVEFRONT_sum" \
           "TA_BUFFER_COALESCED_WRITE_CYCLES_sum TA_BUFFER_COALESCED_READ_CYCLES_sum TD_TD_BUSY_sum TD_SPI_STALL_sum" \
           "TA_BUFFER_TOTAL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum" ; do
  i=$((i+1))
  timeout -k 5 -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -T --kernel-include-regex "pyr_tri" -d $OUT/p$i -o run --output-format csv -- \
    python3 tools/stage_bench.py --reps 1 --fast > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $OUT > $OUT/table.txt && head -30 $OUT/table.txt
