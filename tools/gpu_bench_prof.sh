#!/bin/bash
# bench + rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python bench.py --steps 20 --warmup 2 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
echo done
