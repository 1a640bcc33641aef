set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -k "descriptor or golden or batch" > gpurun_out/ab_tests.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --tag v2 > gpurun_out/ab.log 2>&1 &&
SIFT_HIP_DESC_V1=1 timeout -k 10 120 python tools/stage_bench.py --tag v1 >> gpurun_out/ab.log 2>&1
echo "exit $?"
