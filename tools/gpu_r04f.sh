#!/bin/bash
# round-4 dev pass: gang / Harder / walker teacher-forced tests; A/B of the round-3 tree against
# this tree on every step kernel of the metric robots.  usage: tools/gpu_r04f.sh TAG
set -o pipefail
TAG=${1:-r04f}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gang or Harder or quad or teacher_forced_parity" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python tools/ab_lib.py ab/r03 pybullet-gym_amd/libpbg_amd.so AntPyBulletEnv-v0:16384 HumanoidPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 Walker2DPyBulletEnv-v0:4096 HopperPyBulletEnv-v0:4096 > $OUT/ab_r03.txt 2>&1; rc=$?
cat $OUT/ab_r03.txt
exit $rc
