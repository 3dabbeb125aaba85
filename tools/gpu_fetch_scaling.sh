#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the gang step kernels at two env counts (is the
# read excess per launch -- code / tables -- or per env?).  usage: tools/gpu_fetch_scaling.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
OUT=$R/gpurun_out/${1:-fetchscale}; mkdir -p $OUT
export TMPDIR=/tmp
for W in Hopper:4096 Hopper:16384 Humanoid:4096 Humanoid:16384 Ant:16384 Ant:65536; do
  E=${W%%:*}; N=${W#*:}
  B="python bench.py --steps 20 --warmup 2 --no-cpu-baseline --legs none --precision 32 --env ${E}PyBulletEnv-v0 --envs-per-gpu $N"
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${E}_$N/fetch -o run -- $B > $OUT/${E}_$N.fetch.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${E}_$N/write -o run -- $B > $OUT/${E}_$N.write.log 2>&1 || exit 1
done
echo fetch scaling done
