#!/bin/bash
# Round-3 GPU pass: full -m gpu suite with the parity report, smoke, bench.  usage: tools/gpu_r03.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${1:-r03a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rm -f $OUT/parity.jsonl
PBG_PARITY_DUMP=$OUT/dump PBG_PARITY_REPORT=$OUT/parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1
rc=$?
tail -3 $OUT/gpu_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
exit $rc
