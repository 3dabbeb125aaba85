#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes over tools/fetch_calib (known byte counts per access
# shape).  usage: tools/gpu_fetch_calib.sh TAG   then python tools/fetch_calib_summary.py gpurun_out/TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${1:-calib}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- ./tools/fetch_calib > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- ./tools/fetch_calib > $OUT/write.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/pmc_req -o run -- ./tools/fetch_calib > $OUT/req.log 2>&1 || exit 1
echo calib done
