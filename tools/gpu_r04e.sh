#!/bin/bash
# round-4 dev pass: gang / Harder / Atlas tests; A/B of the round-3 tree against this tree; A/B of
# ab/base.so (same tree without the last change) against this tree.  usage: tools/gpu_r04e.sh TAG
set -o pipefail
TAG=${1:-r04e}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gang or Harder or (teacher_forced_parity and (Atlas or Humanoid or Walker or Cheetah))" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_lib.py ab/base.so pybullet-gym_amd/libpbg_amd.so HalfCheetahPyBulletEnv-v0:8192 HumanoidPyBulletEnv-v0:4096 Walker2DPyBulletEnv-v0:4096 HopperPyBulletEnv-v0:4096 > $OUT/ab_prefetch.txt 2>&1; rc=$?
cat $OUT/ab_prefetch.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/ab_lib.py ab/r03 pybullet-gym_amd/libpbg_amd.so HumanoidPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 Walker2DPyBulletEnv-v0:4096 HopperPyBulletEnv-v0:4096 HumanoidFlagrunHarderPyBulletEnv-v0:4096 AtlasPyBulletEnv-v0:4096 > $OUT/ab_r03.txt 2>&1; rc=$?
cat $OUT/ab_r03.txt
exit $rc
