# A/B of descriptor variants: parity subset, then stage timings of each
# variant on the same device (env switches read by libsift_hip.so).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "descriptor or golden or batch" > gpurun_out/ab_tests.log 2>&1 &&
SIFT_HIP_DESC_PERM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "golden" >> gpurun_out/ab_tests.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --tag scatter > gpurun_out/ab.log 2>&1 &&
SIFT_HIP_DESC_PERM=1 timeout -k 10 120 python tools/stage_bench.py --tag perm >> gpurun_out/ab.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --tag scatter2 >> gpurun_out/ab.log 2>&1
echo "exit $?"
