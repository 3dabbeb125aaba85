#!/bin/bash
# Stall / LDS PMC passes for the two metric workloads (one rocprofv3 run per pass).
# usage: tools/gpu_stalls.sh TAG
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
TAG=${1:-stalls}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for W in ${PROF_ROBOTS:-ant humanoid ant_f64 humanoid_f64}; do
  case $W in
    ant) A="--env AntPyBulletEnv-v0 --envs-per-gpu 16384 --precision 32";;
    humanoid) A="--env HumanoidPyBulletEnv-v0 --envs-per-gpu 4096 --precision 32";;
    hopper) A="--env HopperPyBulletEnv-v0 --envs-per-gpu 4096 --precision 32";;
    halfcheetah) A="--env HalfCheetahPyBulletEnv-v0 --envs-per-gpu 8192 --precision 32";;
    ant_f64) A="--env AntPyBulletEnv-v0 --envs-per-gpu 16384 --precision 64";;
    humanoid_f64) A="--env HumanoidPyBulletEnv-v0 --envs-per-gpu 4096 --precision 64";;
    hopper_f64) A="--env HopperPyBulletEnv-v0 --envs-per-gpu 4096 --precision 64";;
    halfcheetah_f64) A="--env HalfCheetahPyBulletEnv-v0 --envs-per-gpu 8192 --precision 64";;
  esac
  B="python bench.py --steps 20 --warmup 2 --no-cpu-baseline --second-env none $A"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_ANY --output-format csv -d $OUT/$W/pmc_wait -o run -- $B > $OUT/$W.pmc_wait.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC --output-format csv -d $OUT/$W/pmc_lds -o run -- $B > $OUT/$W.pmc_lds.log 2>&1 || exit 1
done
echo stalls done
