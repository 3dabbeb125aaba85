#!/bin/bash
# round-4 dev pass: gang tests; A/B of the round-3 tree on the small robots; phase stamps at one and
# two waves per SIMD (HalfCheetah 4096 / 8192 envs) and on the Humanoid family.
# usage: tools/gpu_r04g.sh TAG
set -o pipefail
TAG=${1:-r04g}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gang or (teacher_forced_parity and (Walker or Cheetah or Hopper))" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_lib.py ab/r03 pybullet-gym_amd/libpbg_amd.so Walker2DPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 HopperPyBulletEnv-v0:4096 > $OUT/ab_r03.txt 2>&1 || exit 1
cat $OUT/ab_r03.txt
timeout -k 10 400 python tools/stamps.py HalfCheetahPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 HumanoidPyBulletEnv-v0:4096 HumanoidFlagrunHarderPyBulletEnv-v0:4096 AntPyBulletEnv-v0:16384 > $OUT/stamps.txt 2>&1; rc=$?
cat $OUT/stamps.txt
exit $rc
