set -o pipefail
export TMPDIR=/tmp
GA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
GB="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM"
GC="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"
i=0
for grp in "$GA" "$GB" "$GC"; do
  i=$((i+1))
  SIFT_HIP_FAST_V1=0 timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -T --kernel-include-regex "pyr_scales|base9" -d gpurun_out/sqv2_$i -o run --output-format csv -- python3 tools/stage_bench.py --reps 1 --fast > gpurun_out/sqv2_$i.log 2>&1 || exit 1
done
