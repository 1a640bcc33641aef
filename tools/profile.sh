#!/bin/bash
# rocprofv3 evidence for one tree (run on the GPU box; every pass is its own
# process, counters never combined with runtime/sys tracing):
#   trace      --kernel-trace --stats over bench.py (exact + fast legs; --streams 1:
#              every launch covers the whole 64-image batch, none overlaps another,
#              so per-launch durations and bytes match bench.py's serial leg)
#   fetch/write  --pmc FETCH_SIZE / WRITE_SIZE over bench.py (one step each)
#   cal_f/cal_w  the same counters over tools/fetch_calib (known byte counts)
#   sqA..sqC   SQ / GRBM / TCC counter groups over tools/stage_bench.py for the
#              named kernels (exact path), sqF* the same for pyr_pc_kernel (SIFT_FLAG_FAST default)
# usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r2}; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="$@"
RE="descriptor_kernel|blur_octave_kernel|blur_sym_kernel|orient_slots_kernel|orient_bin_kernel|extrema_walk_kernel|refine_kernel"
GA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
GB="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM"
GC="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum"
run() {  # name, timeout, rocprof args..., -- cmd
  local name=$1 t=$2; shift 2
  timeout -k 10 -s KILL $t rocprofv3 "$@" > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -5 $OUT/$name.log; exit 1; }
}
timeout -k 5 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
run trace 400 --kernel-trace --stats -T -d $OUT/trace -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-single --no-8k --no-match --streams 1 $ARGS
run fetch 300 --kernel-trace --pmc FETCH_SIZE -T -d $OUT/fetch -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-single --no-8k --no-match --streams 1 --steps 1 --warmup 1 $ARGS
run write 300 --kernel-trace --pmc WRITE_SIZE -T -d $OUT/write -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-single --no-8k --no-match --streams 1 --steps 1 --warmup 1 $ARGS
run cal_f 120 --kernel-trace --pmc FETCH_SIZE -d $OUT/cal_f -o run --output-format csv -- ./tools/fetch_calib
run cal_w 120 --kernel-trace --pmc WRITE_SIZE -d $OUT/cal_w -o run --output-format csv -- ./tools/fetch_calib
i=0
for grp in "$GA" "$GB" "$GC"; do
  i=$((i+1))
  run sq$i 300 --kernel-trace --pmc $grp -T --kernel-include-regex "$RE" -d $OUT/sq$i -o run --output-format csv -- \
    python3 tools/stage_bench.py --reps 1
  run sqF$i 300 --kernel-trace --pmc $grp -T --kernel-include-regex "pyr_pc" -d $OUT/sqF$i -o run --output-format csv -- \
    python3 tools/stage_bench.py --reps 1 --fast
done
run single 200 --kernel-trace --stats -T -d $OUT/single -o run --output-format csv -- \
  python3 tools/single_trace.py --reps 20
echo "profile $TAG done"
