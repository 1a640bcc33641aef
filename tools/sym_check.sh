#!/bin/bash
# GPU check of the scatter-form blur: its parity tests, then a same-box A/B of
# the stage times against the gather-form tiles (SIFT_HIP_BLUR_GATHER=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "scatter or blur_paths or pyramid or golden or batch" > gpurun_out/sym_pytest.log 2>&1 &&
tools/ab_env.sh "SIFT_HIP_BLUR_GATHER=1" "SIFT_HIP_BLUR_GATHER=0" "SIFT_HIP_BLUR_GATHER=1" "SIFT_HIP_BLUR_GATHER=0" \
  > gpurun_out/sym_ab.log 2>&1
rc=$?
tail -5 gpurun_out/sym_pytest.log
cat gpurun_out/sym_ab.log
exit $rc
