#!/bin/bash
# persistent kernels (descriptor, refinement, orientation) sized for half the resident slots (gdiv2) vs all (gref),
# exact headline leg with its 2 sub-batch streams
set -o pipefail
mkdir -p gpurun_out
R=3 bash tools/ab_bench_lib.sh gref gdiv2 2>&1 | tee gpurun_out/r4_griddiv_bench.txt || exit 1
