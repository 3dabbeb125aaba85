#!/bin/bash
# Round-4 GPU pass: the gang-kernel tests first (fail fast), the full -m gpu suite with the parity
# report, smoke, bench, and a Humanoid 16- vs 32-lane bench.  usage: tools/gpu_r04.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${1:-r04a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rm -f $OUT/parity.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "gang or free_running" > $OUT/gang_tests.txt 2>&1
rc=$?
tail -3 $OUT/gang_tests.txt
[ $rc -eq 0 ] || exit $rc
PBG_PARITY_DUMP=$OUT/dump PBG_PARITY_REPORT=$OUT/parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?
tail -3 $OUT/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
for L in 16 32; do
  timeout -k 10 120 python bench.py --env HumanoidPyBulletEnv-v0 --envs-per-gpu 4096 --legs none --no-cpu-baseline --gang-lanes $L > $OUT/bench_humanoid_$L.json 2>> $OUT/bench.err || exit 1
done
cat $OUT/bench.json | head -c 600; echo
grep -o '"kernel_ms": [0-9.e-]*' $OUT/bench_humanoid_*.json
exit $rc
