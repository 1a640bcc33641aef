#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=3 bash tools/ab_var.sh r4abl2 prod abl8 abl1 || exit 1
