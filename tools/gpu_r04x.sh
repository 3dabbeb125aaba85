#!/bin/bash
# round-4 dev pass: XCD-aware env block order -- tests, A/B, HBM traffic passes (Ant, Humanoid)
set -o pipefail
TAG=${1:-r04x}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "gang or quad or teacher_forced_parity or determinism or shard or checkpoint or reset" > $OUT/tests.txt 2>&1; rc=$?
tail -3 $OUT/tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python tools/ab_lib.py ab/base.so ab/new.so AntPyBulletEnv-v0:16384 HumanoidPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 HopperPyBulletEnv-v0:4096 > $OUT/ab.txt 2>&1 || exit 1
cat $OUT/ab.txt
for W in ant humanoid; do
  if [ $W = ant ]; then A="--env AntPyBulletEnv-v0 --envs-per-gpu 16384"; else A="--env HumanoidPyBulletEnv-v0 --envs-per-gpu 4096"; fi
  B="python bench.py --steps 20 --warmup 2 --no-cpu-baseline --second-env none $A"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$W/pmc_fetch -o run -- $B > $OUT/$W.pmc_fetch.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$W/pmc_write -o run -- $B > $OUT/$W.pmc_write.log 2>&1 || exit 1
done
echo traffic done
