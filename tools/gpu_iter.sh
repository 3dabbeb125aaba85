#!/bin/bash
# dev loop on the GPU box: gpu tests, throughput table, phase stamps
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${1:-it}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/$TAG/tests.log 2>&1; rc=$?; echo "tests rc=$rc" >> gpurun_out/$TAG/tests.log
# a fault / abort / timeout ends the GPU work of this call
case $rc in 124|134|137|139) tail -5 gpurun_out/$TAG/tests.log; exit $rc;; esac
timeout -k 10 200 python tools/throughput.py > gpurun_out/$TAG/throughput.log 2>&1 && \
timeout -k 10 200 python tools/stamps.py AntPyBulletEnv-v0:16384 HumanoidPyBulletEnv-v0:4096 > gpurun_out/$TAG/stamps.log 2>&1
tail -3 gpurun_out/$TAG/tests.log; cat gpurun_out/$TAG/throughput.log
