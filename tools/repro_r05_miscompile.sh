#!/bin/bash
# Reproduces the round-5 float64 quad miscompile's faulting ISA from git history:
# compiles the round-5 source (commit 4428492) of team_step_kernel<F64<Ant>,16> under the default machine
# schedule and under the register-pressure trackers, then runs the partial-EXEC copy check on both.
# Expected: the default build has the VGPR->AGPR split copies of a54/a55/a180/a181 in a divergent
# region's join block before its EXEC restore (plus one harmless re-copy); the trackers build has none.
# CPU only.  usage: tools/repro_r05_miscompile.sh [WORKDIR]
set -euo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
W=${1:-/tmp/pbg_r05_repro}
rm -rf "$W" && mkdir -p "$W"
git -C "$REPO" archive 44284927f8c7b1aa8bfb3a2ce5060a444b8317e4 pybullet-gym_amd/csrc include | tar -x -C "$W"
F="--offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DPBG_TEAM64_TU -DPBG_ROBOT=Ant --cuda-device-only -S"
cd "$W/pybullet-gym_amd"
/opt/rocm/bin/hipcc $F -o "$W/default.s" csrc/pbg_robot.hip 2> /dev/null &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-use-amdgpu-trackers=1 -o "$W/trackers.s" csrc/pbg_robot.hip 2> /dev/null &
wait
python3 "$REPO/tools/isa_uninit.py" "$W/default.s" --exec-copies || true
python3 "$REPO/tools/isa_uninit.py" "$W/trackers.s" --exec-copies
