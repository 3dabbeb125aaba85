set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r02c/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/r02c/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r02c/gpu_tests.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02c/smoke.txt 2>&1 || { cat gpurun_out/r02c/smoke.txt; exit 1; }
bash tools/gpu_bench_prof.sh r02c || exit 1
bash tools/gpu_stalls.sh r02c || exit 1
cat gpurun_out/r02c/bench.json
