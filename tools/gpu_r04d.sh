#!/bin/bash
# round-4 dev pass: gang / Harder / Atlas tests, then an A/B of the round-3 tree (ab/r03) against
# this tree on the gang robots.  usage: tools/gpu_r04d.sh TAG
set -o pipefail
TAG=${1:-r04d}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gang or Harder or (teacher_forced_parity and (Atlas or Humanoid))" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/ab_lib.py ab/r03 pybullet-gym_amd/libpbg_amd.so HumanoidPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 Walker2DPyBulletEnv-v0:4096 HopperPyBulletEnv-v0:4096 HumanoidFlagrunHarderPyBulletEnv-v0:4096 AtlasPyBulletEnv-v0:4096 > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt
exit $rc
