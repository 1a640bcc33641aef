set -o pipefail
mkdir -p gpurun_out
[ "$SKIP_CHECK" = 1 ] || bash tools/gpu_check.sh r5j || exit 1
L=sift-gpu_amd/lib
cp $L/libsift_hip.so $L/libsift_hip_keep8k.so
for v in cur pcabl1 pcabl3 pcabl48 pcabl51; do
  [ $v = cur ] || cp $L/libsift_hip_$v.so $L/libsift_hip.so
  timeout -k 10 300 python3 bench.py --only 8k --steps 5 --warmup 2 > gpurun_out/r5j_8k_$v.json 2> gpurun_out/r5j_8k_$v.err || { echo "8k $v failed"; tail -3 gpurun_out/r5j_8k_$v.err; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['image_8k']['roofline']['fast_pyramid']; print(sys.argv[2], r['ms_per_image'], r['frac'])" gpurun_out/r5j_8k_$v.json $v
  cp $L/libsift_hip_keep8k.so $L/libsift_hip.so
done
R=2 bash tools/ab.sh fast r5jabl cur pcabl1 pcabl3 pcabl48 pcabl51
