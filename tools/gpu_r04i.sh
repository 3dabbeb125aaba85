#!/bin/bash
# round-4 profile pass: bench + rocprof kernel stats + PMC passes (four bench workloads), stall /
# LDS passes (Ant, Humanoid), HumanoidFlagrunHarder contact-count histogram.  usage: TAG
set -o pipefail
TAG=${1:-r04i}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_bench_prof.sh $TAG --steps 1000 --warmup 50 || exit 1
bash tools/gpu_stalls.sh ${TAG}_stalls || exit 1
timeout -k 10 200 python tools/contact_hist.py HumanoidFlagrunHarderPyBulletEnv-v0:4096 HumanoidPyBulletEnv-v0:4096 > $OUT/contact_hist.txt 2>&1 || exit 1
cat $OUT/contact_hist.txt
