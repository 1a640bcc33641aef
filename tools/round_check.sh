set -o pipefail
bash tools/gpu_check.sh && bash tools/profile.sh r1b --steps 5 --warmup 2
