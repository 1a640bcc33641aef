#!/bin/bash
# rocprofv3 over the SIFT_FLAG_FAST pyramid kernels (tools/stage_bench.py --fast):
# kernel trace + stats, then SQ / GRBM / TCC counter passes, each its own run.
# usage: tools/prof_fast.sh <tag> [regex]
set -o pipefail
TAG=${1:-fast}; RE=${2:-pyr_pair|pyr_fast}
O=gpurun_out/pf_$TAG
mkdir -p $O
export TMPDIR=/tmp
run() {  # name, timeout, rocprof args...
  local name=$1 t=$2; shift 2
  timeout -k 10 -s KILL $t rocprofv3 "$@" -- python3 tools/stage_bench.py --fast --reps 2 > $O/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $O/$name.log; exit 1; }
}
run trace 240 --kernel-trace --stats -T -d $O/trace -o run --output-format csv
run sq1 240 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU -T --kernel-include-regex "$RE" -d $O/sq1 -o run --output-format csv
run sq2 240 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -T --kernel-include-regex "$RE" -d $O/sq2 -o run --output-format csv
run gr 240 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -T --kernel-include-regex "$RE" -d $O/gr -o run --output-format csv
run fe 240 --kernel-trace --pmc FETCH_SIZE -T --kernel-include-regex "$RE" -d $O/fe -o run --output-format csv
run wr 240 --kernel-trace --pmc WRITE_SIZE -T --kernel-include-regex "$RE" -d $O/wr -o run --output-format csv
[ -n "$ICACHE" ] && run ic 240 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -T --kernel-include-regex "$RE" -d $O/ic -o run --output-format csv
echo "prof_fast $TAG done"
