#!/bin/bash
# SQ / GRBM / TA / TD counter passes over tools/stage_bench.py for the kernels
# matching a regex, one rocprofv3 process per group (kernel-trace only beside
# the counters), optionally for several library builds; pmc_table.py turns
# each run into a table.  Replaces pmc_kernel.sh / pmc_lib.sh / pmc_tri.sh.
# usage: tools/pmc.sh <tag> <kernel regex> [<lib name>...]   (MODE=fast: SIFT_FLAG_FAST;
#        PMC_SETS=sq|mem|all, default sq; PROG="<script + args>" instead of tools/stage_bench.py,
#        e.g. PROG="tools/single_trace.py --reps 3" for the one-image kernels)
set -o pipefail
TAG=$1; RE=$2; shift 2
[ -n "$TAG" ] && [ -n "$RE" ] || { sed -n '2,8p' "$0"; exit 2; }
L=sift-gpu_amd/lib
export TMPDIR=/tmp
FL=; [ "$MODE" = fast ] && FL=--fast
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_SALU"
SQ3="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_WR"
MEM="TA_TA_BUSY_sum TA_BUFFER_WRITE_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_WRITE_REQ_LATENCY_sum"
case ${PMC_SETS:-sq} in
  sq) SETS=("$SQ1" "$SQ2") ;;
  mem) SETS=("$SQ3" "$MEM") ;;
  all) SETS=("$SQ1" "$SQ2" "$SQ3" "$MEM") ;;
esac
[ $# -eq 0 ] && set -- cur
cp $L/libsift_hip.so $L/libsift_hip_pmckeep.so
trap 'cp $L/libsift_hip_pmckeep.so $L/libsift_hip.so' EXIT
for n in "$@"; do
  [ "$n" = cur ] || cp $L/libsift_hip_$n.so $L/libsift_hip.so
  OUT=gpurun_out/pmc_${TAG}_$n
  mkdir -p $OUT
  i=0
  for grp in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 5 -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -T --kernel-include-regex "$RE" -d $OUT/p$i -o run \
      --output-format csv -- python3 ${PROG:-tools/stage_bench.py --reps 1 --ignore-status $FL} > $OUT/p$i.log 2>&1 \
      || { echo "pass $n $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  python3 tools/pmc_table.py $OUT > $OUT/table.txt
  echo "== $n"; head -30 $OUT/table.txt
  [ "$n" = cur ] || cp $L/libsift_hip_pmckeep.so $L/libsift_hip.so
done
