#!/bin/bash
# round-4 dev pass: quad-kernel tests, A/B of ab/base.so vs ab/new.so on the Ant
set -o pipefail
TAG=${1:-r04n}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "Ant or quad or workspace" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_lib.py ab/base.so ab/new.so AntPyBulletEnv-v0:16384 AntPyBulletEnv-v0:16384 > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt
exit $rc
