#!/bin/bash
# ablations (timing only, garbage descriptors): chain reads before writes; no gather (constant pixel); no value stores
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MODE=exact R=2 bash tools/ab_var.sh r4nochain dref dnochain dnogather dnostash || exit 1
