#!/bin/bash
# Per-launch durations of the scatter and gather blurs (kernel trace), then SQ
# counter passes over blur_sym_kernel.  usage: tools/sym_prof.sh <tag>
set -o pipefail
TAG=${1:-sym}
OUT=gpurun_out/symprof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace -T -d $OUT/tr_sym -o run --output-format csv -- \
  python3 tools/stage_bench.py --reps 2 > $OUT/tr_sym.log 2>&1 || { echo "trace sym failed"; exit 1; }
SIFT_HIP_BLUR_GATHER=1 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace -T -d $OUT/tr_gat -o run --output-format csv -- \
  python3 tools/stage_bench.py --reps 2 > $OUT/tr_gat.log 2>&1 || { echo "trace gather failed"; exit 1; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --pmc $grp -T --kernel-include-regex "blur_sym|blur_octave|blur_plane" \
    -d $OUT/sq$i -o run --output-format csv -- python3 tools/stage_bench.py --reps 1 > $OUT/sq$i.log 2>&1 \
    || { echo "pass $i failed"; exit 1; }
done
echo done
