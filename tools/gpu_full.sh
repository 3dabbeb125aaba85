set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
mkdir -p gpurun_out/r02e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02e/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r02e/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r02e/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02e/smoke.txt 2>&1 || { cat gpurun_out/r02e/smoke.txt; exit 1; }
bash tools/gpu_bench_prof.sh r02e || exit 1
bash tools/gpu_stalls.sh r02e || exit 1
cat gpurun_out/r02e/bench.json
if [ -f pybullet-gym_amd/libpbg_amd_stamps.so ]; then
  timeout -k 10 200 python tools/stamps.py AntPyBulletEnv-v0:16384 HumanoidPyBulletEnv-v0:4096 HalfCheetahPyBulletEnv-v0:8192 > gpurun_out/r02e/stamps.log 2>&1 || exit 1
fi
