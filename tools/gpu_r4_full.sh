#!/bin/bash
# GPU call: full -m gpu suite, smoke, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4_gpu_tests_full.log 2>&1 || { tail -40 gpurun_out/r4_gpu_tests_full.log; exit 1; }
tail -2 gpurun_out/r4_gpu_tests_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err || { tail -20 gpurun_out/r4_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r4_bench.json').read().strip().splitlines()[-1])
print('value', d['value'], d['ms_per_step'], 'fast', d.get('fast_mode',{}).get('value'), d.get('roofline_pyramid_fast',{}).get('frac'), 'single', d.get('single_image',{}).get('latency_ms'))
print('stages', d.get('stages_ms_per_step'))
"
