#!/bin/bash
# One parameterised GPU pass (replaces the per-call tools/gpu_r0*.sh scripts).
#   tools/gpu_run.sh TAG [STEP ...]      steps run in order, each under its own time limit:
#     tests[:PYTEST_K]  pytest -m gpu (optionally -k PYTEST_K) with the parity report
#     full              the whole -m gpu suite (+ parity report, dumps)
#     smoke             __graft_entry__.smoke()
#     bench[:ARGS]      python bench.py ARGS (ARGS: comma-separated)
#     prof              tools/gpu_bench_prof.sh TAG_prof (bench + rocprof stats + PMC passes)
#     stalls            tools/gpu_stalls.sh TAG_stalls
# A step that faults, aborts or times out ends the call (no later GPU step runs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
nb=0
for S in "$@"; do
  name=${S%%:*}; arg=${S#*:}; [ "$arg" = "$S" ] && arg=""
  echo "== $S $(date +%T)"
  case $name in
    tests)
      K=(); [ -n "$arg" ] && K=(-k "$arg")
      PBG_PARITY_REPORT=$OUT/parity.jsonl timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --timeout 300 \
        --timeout-method thread "${K[@]}" > $OUT/tests_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40).txt 2>&1
      rc=$?; tail -3 $OUT/tests_*.txt | tail -3;;
    full)
      PBG_PARITY_DUMP=$OUT/dump PBG_PARITY_REPORT=$OUT/parity.jsonl timeout -k 10 2400 python -u -m pytest tests -m gpu -v -s \
        --timeout 900 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
      rc=$?; tail -3 $OUT/gpu_tests.txt;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1; rc=$?; tail -2 $OUT/smoke.txt;;
    bench)
      nb=$((nb + 1)); BF=$OUT/bench_${nb}_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40).json
      timeout -k 10 400 python bench.py ${arg//,/ } > $BF 2>> $OUT/bench.err; rc=$?; tail -c 400 $BF;;
    prof)
      bash tools/gpu_bench_prof.sh ${TAG}_prof --steps 1000 --warmup 50; rc=$?;;
    stalls)
      bash tools/gpu_stalls.sh ${TAG}_stalls; rc=$?;;
    *) echo "unknown step $S"; rc=2;;
  esac
  echo "== $S rc=$rc $(date +%T)"
  # pytest exit 1 = test failures (the GPU is fine: go on); anything else ends the call
  [ $rc -eq 0 ] || { [ $name = tests -o $name = full ] && [ $rc -eq 1 ]; } || exit $rc
done
exit $rc
