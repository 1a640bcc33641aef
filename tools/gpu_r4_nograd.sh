#!/bin/bash
# ablation (timing only, wrong descriptors/orientations): extrema walk writes gradients only for strip-edge lanes
set -o pipefail
mkdir -p gpurun_out
MODE=exact R=2 bash tools/ab_var.sh r4nograd xref xnograd || exit 1
R=3 bash tools/ab_bench_lib.sh xref xnograd 2>&1 | tee gpurun_out/r4_nograd_bench.txt || exit 1
