#!/bin/bash
# round-4 dev pass: 32-lane Humanoid gangs with the rows pass reading the factor from LDS
set -o pipefail
TAG=${1:-r04y}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gang" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python tools/ab_lib.py ab/base.so ab/new.so HumanoidPyBulletEnv-v0:4096:-1:32 HumanoidPyBulletEnv-v0:4096:-1:16 HumanoidFlagrunHarderPyBulletEnv-v0:4096:-1:32 > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt
exit $rc
