#!/bin/bash
# round-4 dev pass: reset / quad / gang tests + A/B ab/base.so vs ab/new.so on the bench robots
set -o pipefail
TAG=${1:-r04v}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "reset or autoreset or gang or quad or teacher_forced_parity or checkpoint or determinism" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python tools/ab_lib.py ab/base.so ab/new.so HopperPyBulletEnv-v0:4096 Walker2DPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 AntPyBulletEnv-v0:16384 HumanoidPyBulletEnv-v0:4096 > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt
exit $rc
