#!/bin/bash
# dev loop on the GPU box: gpu tests (optional -k filter), then A/B of ab/base.so against the
# in-tree libpbg_amd.so, then phase stamps when the stamps library exists.
# usage: tools/gpu_ab.sh TAG "pytest -k expr or ''" ENV:N [ENV:N ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${1:-ab}; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ -n "$K" ]; then
  timeout -k 10 ${TT:-400} python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1; rc=$?
  echo "tests rc=$rc" >> $OUT/tests.log; tail -3 $OUT/tests.log
  case $rc in 0|5) ;; *) exit $rc;; esac
fi
timeout -k 10 500 python tools/ab_lib.py ${BASE:-ab/base.so} pybullet-gym_amd/libpbg_amd.so "$@" > $OUT/ab.log 2>&1; rc=$?
cat $OUT/ab.log; [ $rc = 0 ] || exit $rc
if [ -f pybullet-gym_amd/libpbg_amd_stamps.so ]; then
  timeout -k 10 200 python tools/stamps.py "$@" > $OUT/stamps.log 2>&1; rc=$?; cat $OUT/stamps.log; exit $rc
fi
