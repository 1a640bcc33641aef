#!/bin/bash
# orientation: two gather buffers, two batches ahead, no latch copies (o1) vs
# the committed loop (o0); descriptor: PF = 2 gather pinned ahead of the chain
# + prologue flush (o1) vs without (d1).  Full GPU suite on the candidate first.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r4_o2_tests.log 2>&1 || { tail -30 gpurun_out/r4_o2_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r4_o2_tests.log)"
MODE=exact R=2 bash tools/ab_var.sh r4o2 o0 o1 d1 || exit 1
R=2 bash tools/ab_bench_lib.sh o0 o1 d1 2>&1 | tee gpurun_out/r4_o2_bench.txt || exit 1
R=2 bash tools/ab_single.sh o0 o1 || exit 1
