#!/bin/bash
# bench + rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE; WRITE_SIZE; SQ
# instruction/cycle counters; VALU op mix) for the bench workloads (Ant 16,384 envs, Humanoid
# 4,096, Hopper 4,096, HalfCheetah 8,192; PROF_ROBOTS="ant humanoid" narrows the list).  usage: tools/gpu_bench_prof.sh TAG [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
shift || true
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
# the bench command itself (same steps / warmup), without the CPU leg
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python bench.py --no-cpu-baseline "$@" > $OUT/trace.log 2>&1
for W in ${PROF_ROBOTS:-ant humanoid hopper halfcheetah ant_f64 humanoid_f64 hopper_f64 halfcheetah_f64}; do
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
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$W/pmc_fetch -o run -- $B > $OUT/$W.pmc_fetch.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$W/pmc_write -o run -- $B > $OUT/$W.pmc_write.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/$W/pmc_sq -o run -- $B > $OUT/$W.pmc_sq.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_INT32 --output-format csv -d $OUT/$W/pmc_flops -o run -- $B > $OUT/$W.pmc_flops.log 2>&1
  # L2 hit / miss and L1->L2 reads (is the gang kernels' read excess the tables?)
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/$W/pmc_l2 -o run -- $B > $OUT/$W.pmc_l2.log 2>&1
  case $W in *_f64) timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FLOPS_FP64 --output-format csv -d $OUT/$W/pmc_flops64 -o run -- $B > $OUT/$W.pmc_flops64.log 2>&1;; esac
done
echo done
