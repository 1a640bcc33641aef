#!/bin/bash
# One GPU call's closing check of the current tree: the -m gpu suite, smoke(),
# the default bench line, and (PROFILE=1) the rocprofv3 passes of
# tools/profile.sh.  Replaces final_r3.sh / final_r4.sh / gpu_r4_check.sh.
# usage: tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-check}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
  || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed rc=$?"; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms', d['ms_per_step'], 'verified', d['output_verified'], 'desc', d['stages_ms_per_step'].get('descriptor'))
print('fast', (d.get('fast_mode') or {}).get('value'), 'frac', (d.get('roofline_pyramid_fast') or {}).get('frac'),
      'single', (d.get('single_image') or {}).get('latency_ms'), '8k', (d.get('image_8k') or {}).get('latency_ms'))
"
if [ "${PROFILE:-0}" = 1 ]; then bash tools/profile.sh $TAG || exit 1; fi
echo "check $TAG done"
