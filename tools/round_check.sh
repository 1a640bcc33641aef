#!/bin/bash
# Round-end GPU check: smoke, the -m gpu suite, a short bench, then the
# rocprofv3 passes of tools/profile.sh under the given tag.
#   tools/round_check.sh <tag>
set -o pipefail
bash tools/gpu_check.sh && bash tools/profile.sh ${1:-r1c} --steps 5 --warmup 2
