#!/bin/bash
# -m gpu suite, smoke() and the default bench line on the current library.
set -o pipefail
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value',d['value'],'ms',d['ms_per_step'],'desc',d['stages_ms_per_step']['descriptor'])
for k in ('single_image','fast','image_8k'):
    v=d.get(k)
    if isinstance(v,dict): print(k, {kk:vv for kk,vv in v.items() if not isinstance(vv,(dict,list))})
"
