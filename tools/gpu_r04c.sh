set -o pipefail
OUT=gpurun_out/r04c; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "(teacher_forced_parity and Atlas) or (policy_device and Walker2D)" > $OUT/tests.txt 2>&1; rc=$?; tail -3 $OUT/tests.txt
timeout -k 10 300 python tools/stamps.py HumanoidPyBulletEnv-v0:4096:-1:16 HumanoidPyBulletEnv-v0:4096:-1:32 HalfCheetahPyBulletEnv-v0:8192 > $OUT/stamps.txt 2>&1 || exit 1
cat $OUT/stamps.txt
for E in AtlasPyBulletEnv-v0:4096 Walker2DPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 HopperPyBulletEnv-v0:4096; do
  timeout -k 10 200 python bench.py --env ${E%%:*} --envs-per-gpu ${E##*:} --legs none --no-cpu-baseline --steps 200 --windows 3 > $OUT/bench_${E%%:*}.json 2>>$OUT/bench.err || exit 1
  grep -o '"kernel_ms": [0-9.e-]*' $OUT/bench_${E%%:*}.json | head -1
done
exit $rc
