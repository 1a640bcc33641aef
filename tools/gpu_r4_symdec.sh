#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_symdec_tests.log 2>&1 || { tail -30 gpurun_out/r4_symdec_tests.log; exit 1; }
tail -1 gpurun_out/r4_symdec_tests.log
MODE=exact R=2 bash tools/ab_var.sh r4symdec base symdec || exit 1
R=3 bash tools/ab_bench_lib.sh base symdec 2>&1 | tee gpurun_out/r4_symdec_bench.txt || exit 1
R=2 bash tools/ab_single.sh base symdec || exit 1
