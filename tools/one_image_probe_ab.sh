for r in 1 2; do
for sz in "2160 3840" "1440 2560" "3072 4096"; do
  for lim in default 0 100000000; do
    if [ $lim = default ]; then E=""; else E="SIFT_HIP_ONE_IMAGE_PX=$lim"; fi
    env $E timeout -k 10 120 python3 tools/one_image_probe.py $sz --tag "$lim" || exit 1
  done
done
done
