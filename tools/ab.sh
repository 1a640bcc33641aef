#!/bin/bash
# Same-box A/B of library builds or library environment settings, alternating,
# R rounds (default 2).  One script for every A/B in DESIGN.md since round 5
# (it replaces the per-experiment gpu_r4_*.sh wrappers).
#
# usage: tools/ab.sh <leg> <tag> <variant>...
#   leg      fast    tools/stage_bench.py --fast: the SIFT_FLAG_FAST pyramid stage times
#            exact   tools/stage_bench.py: every exact-path stage time
#            bench   bench.py's exact headline leg (2 streams, graph replay, --steps 10)
#            single  bench.py's configs[1] one-image leg
#            8k      bench.py's configs[4] leg (one 8K image: exact latency + fast-pyramid roofline)
#   variant  <name>            lib/libsift_hip_<name>.so (tools/build_var.sh, tools/build_patch.sh);
#                              "cur" = the current lib/libsift_hip.so
#            VAR=val[,VAR=val] the current build with those environment settings
# env:  R      rounds (default 2)
#       TESTS  pytest -k expression: those -m gpu tests run once per library variant first
#       ARGS   extra arguments for the timed command
# Output: gpurun_out/ab_<tag>/ (raw logs) and one summary line per run on stdout.
set -o pipefail
LEG=$1; TAG=$2; shift 2
[ -n "$LEG" ] && [ -n "$TAG" ] && [ $# -ge 1 ] || { sed -n '2,20p' "$0"; exit 2; }
export TMPDIR=/tmp
L=sift-gpu_amd/lib
O=gpurun_out/ab_$TAG
mkdir -p $O
cp $L/libsift_hip.so $L/libsift_hip_abkeep.so
restore() { cp $L/libsift_hip_abkeep.so $L/libsift_hip.so; }
trap restore EXIT

select_variant() {  # sets ENVS for an env variant, swaps the library for a build variant
  ENVS=""
  case "$1" in
    *=*) ENVS=$(echo "$1" | tr ',' ' '); restore ;;
    cur) restore ;;
    *) [ -f $L/libsift_hip_$1.so ] || { echo "no $L/libsift_hip_$1.so"; exit 1; }
       cp $L/libsift_hip_$1.so $L/libsift_hip.so ;;
  esac
}

if [ -n "$TESTS" ]; then
  for v in "$@"; do
    case "$v" in *=*) continue ;; esac
    select_variant "$v"
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$TESTS" \
      > $O/tests_$v.log 2>&1 || { echo "tests failed on $v"; tail -30 $O/tests_$v.log; exit 1; }
    echo "tests $v: $(tail -1 $O/tests_$v.log)"
  done
fi

for r in $(seq ${R:-2}); do
  for v in "$@"; do
    select_variant "$v"
    f=$O/$(echo "$v" | tr '=,/' '__-')_$r
    case $LEG in
      fast|exact)
        FL=; [ $LEG = fast ] && FL=--fast
        env $ENVS timeout -k 10 180 python3 tools/stage_bench.py $FL --reps 3 --ignore-status --tag "$v" $ARGS \
          > $f.txt 2>&1 || { echo "run $v failed"; tail -5 $f.txt; exit 1; }
        grep -h "^{" $f.txt | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['tag'], d['total_ms'], json.dumps(d['stages_ms']))" ;;
      bench)
        env $ENVS timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-single --no-8k --no-match --no-fast \
          --steps 10 $ARGS > $f.json 2> $f.err || { echo "bench $v failed"; tail -5 $f.err; exit 1; }
        python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d['ms_per_step'], 'serial', d['serial_leg']['ms_per_step'], 'verified', d['output_verified'],
      'desc', d['stages_ms_per_step'].get('descriptor'))" $f.json "$v" ;;
      single)
        env $ENVS timeout -k 10 300 python3 bench.py --only single --steps 20 --warmup 5 $ARGS > $f.json 2> $f.err \
          || { echo "single $v failed"; tail -5 $f.err; exit 1; }
        python3 -c "
import json, sys
s = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]).get('single_image') or {}
print(sys.argv[2], s.get('latency_ms'), s.get('device_no_graph_ms'), 'verified', s.get('output_verified'))" $f.json "$v" ;;
      8k)
        env $ENVS timeout -k 10 200 python3 bench.py --only 8k --steps 5 --warmup 2 $ARGS > $f.json 2> $f.err \
          || { echo "8k $v failed"; tail -5 $f.err; exit 1; }
        python3 -c "
import json, sys
e = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])['image_8k']
r = e['roofline']
print(sys.argv[2], 'latency_ms', e['latency_ms'], 'blur_ms', r['exact_blur_octave']['ms_per_image'], 'fast_pyr_ms',
      r['fast_pyramid']['ms_per_image'], 'frac', r['fast_pyramid']['frac'], 'verified', e['output_verified'])" $f.json "$v" ;;
      *) echo "unknown leg $LEG"; exit 2 ;;
    esac
  done
done
