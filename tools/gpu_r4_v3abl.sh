#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=2 bash tools/ab_var.sh r4v3abl v3 v3a1 v3a3 v3a16 v3a19 || exit 1
bash tools/pmc_tri.sh tri4v3 > /dev/null || exit 1
grep -A1 "clock_GHz" gpurun_out/pmc_tri4v3/table.txt | head -4
grep "grid" gpurun_out/pmc_tri4v3/table.txt
