#!/bin/bash
# round-4 profile pass on the final kernels: bench + rocprof kernel stats + PMC passes (four bench
# workloads), stall / LDS passes (Ant, Humanoid), phase stamps.  usage: tools/gpu_r04p.sh TAG
set -o pipefail
TAG=${1:-r04p}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_bench_prof.sh $TAG --steps 1000 --warmup 50 || exit 1
bash tools/gpu_stalls.sh ${TAG}_stalls || exit 1
timeout -k 10 400 python tools/stamps.py AntPyBulletEnv-v0:16384 HumanoidPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 HumanoidFlagrunHarderPyBulletEnv-v0:4096 Walker2DPyBulletEnv-v0:4096 HopperPyBulletEnv-v0:4096 > $OUT/stamps.txt 2>&1 || exit 1
tail -20 $OUT/stamps.txt
