# Descriptor iteration: parity subset (descriptor / golden / batch), then two
# exact-mode stage timings.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "descriptor or golden or batch" > gpurun_out/q_tests.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --tag a > gpurun_out/q.log 2>&1 &&
timeout -k 10 120 python tools/stage_bench.py --tag b >> gpurun_out/q.log 2>&1
echo "exit $?"
