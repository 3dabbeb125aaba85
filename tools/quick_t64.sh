#!/bin/bash
# Dev helper: rebuild only the float64 quad kernel's translation unit (team64_Ant, product flags) and link
# it with the product's other objects into pybullet-gym_amd/libpbg_<TAG>.so (an A/B variant of the
# headline kernel in ~2 min instead of a full rebuild).  EXTRA: additional hipcc flags.
#   tools/quick_t64.sh TAG [EXTRA...]
set -e
cd "$(dirname "$0")/../pybullet-gym_amd"
TAG=$1; shift
mkdir -p build/obj_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -DPBG_TEAM64_TU \
  "$@" -DPBG_ROBOT=Ant -c -o build/obj_var/team64_Ant_$TAG.o csrc/pbg_robot.hip
objs=$(ls build/obj/*.o | grep -v "/team64_Ant.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o libpbg_$TAG.so build/obj_var/team64_Ant_$TAG.o $objs
echo built libpbg_$TAG.so
