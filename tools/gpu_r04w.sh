#!/bin/bash
# round-4 final pass: full -m gpu suite + parity report, smoke, bench, then the profile pass
set -o pipefail
TAG=${1:-r04w}
bash tools/gpu_r04.sh $TAG || exit 1
bash tools/gpu_r04p.sh ${TAG}p || exit 1
