#!/bin/bash
# round-4 dev pass: gang tests + A/B ab/base.so vs ab/new.so (Humanoid, Harder, Atlas)
set -o pipefail
TAG=${1:-r04t}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gang or teacher_forced_parity or harder or workspace" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_lib.py ab/base.so ab/new.so HumanoidPyBulletEnv-v0:4096 HumanoidFlagrunHarderPyBulletEnv-v0:4096 AtlasPyBulletEnv-v0:4096 > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt
exit $rc
