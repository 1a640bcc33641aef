#!/bin/bash
# SQ/GRBM counter passes for the kernels matching $2 over tools/stage_bench.py,
# with lib/libsift_hip_<name>.so swapped in for each name.
# usage: tools/pmc_lib.sh <tag> <regex> <name>... (MODE=fast: SIFT_FLAG_FAST)
set -o pipefail
TAG=$1; RE=$2; shift 2
L=sift-gpu_amd/lib
export TMPDIR=/tmp
FL=; [ "$MODE" = fast ] && FL=--fast
cp $L/libsift_hip.so $L/libsift_hip_keep.so
for n in "$@"; do
  cp $L/libsift_hip_$n.so $L/libsift_hip.so
  OUT=gpurun_out/pmc_${TAG}_$n
  mkdir -p $OUT
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -k 5 -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -T --kernel-include-regex "$RE" -d $OUT/p$i -o run --output-format csv -- \
      python3 tools/stage_bench.py --reps 1 --ignore-status $FL > $OUT/p$i.log 2>&1 || { echo "pass $n $i failed"; tail -5 $OUT/p$i.log; cp $L/libsift_hip_keep.so $L/libsift_hip.so; exit 1; }
  done
  python3 tools/pmc_table.py $OUT > $OUT/table.txt
  echo "== $n"; grep -A0 "grid\|clock" $OUT/table.txt | head -4
done
cp $L/libsift_hip_keep.so $L/libsift_hip.so
