set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do for v in 4096 8192 16384 32768 65536; do
  SIFT_HIP_EXTREMA_WAVES=$v timeout -k 10 120 python3 tools/stage_bench.py --reps 5 --tag "W=$v" >> gpurun_out/ab_ew.log 2>/dev/null || exit 1
done; done
grep -h stages_ms gpurun_out/ab_ew.log | python3 -c "
import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['tag'], d['stages_ms']['extrema'], d['total_ms'])"
