#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r6g
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_multi.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6g/pytest.log 2>&1 || { tail -40 gpurun_out/r6g/pytest.log; exit 1; }
tail -1 gpurun_out/r6g/pytest.log
timeout -k 10 400 python -u bench.py --only multi --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r6g/bench_multi.json 2> gpurun_out/r6g/bench_multi.err || { tail -20 gpurun_out/r6g/bench_multi.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r6g/bench_multi.json').read().strip().splitlines()[-1]); print(d.get('c_abi_multi'), d.get('leg_errors'))"
timeout -k 10 400 python -u bench.py --only exact --no-cpu-baseline --no-match --steps 10 --warmup 3 > gpurun_out/r6g/bench_exact.json 2> gpurun_out/r6g/bench_exact.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r6g/bench_exact.json').read().strip().splitlines()[-1]); print('exact', d['value'], d['ms_per_step'])"
