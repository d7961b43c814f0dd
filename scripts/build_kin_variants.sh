#!/bin/bash
# A/B builds of the kinematic kernel: libvcmpc_<tag>.so (and a timing build
# libvcmpc_timing_<tag>.so) with kin_ltv.hip compiled under extra -D flags, every other
# object shared with the default build.  Use them through VCMPC_LIB=...
# usage: bash scripts/build_kin_variants.sh tag "-DFLAG=.." [tag "-D.." ...]
set -e
cd "$(dirname "$0")/../vehicle-control_amd/csrc"
make -j8 >/dev/null
make timing -j8 >/dev/null
HIPCC=/opt/rocm/bin/hipcc
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. -Wall -Wno-unused-function"
OTHER="build/vcmpc_abi.o build/kin_ric.o build/kin_merit.o build/dyn_sqp.o build/casc_sqp.o build/casc_ric.o build/st_sqp.o build/models.o build/track.o build/numerics.o"
OTHER_T="build/vcmpc_abi_timing.o build/kin_ric_timing.o build/kin_merit.o build/dyn_sqp_timing.o build/casc_sqp_timing.o build/casc_ric_timing.o build/st_sqp_timing.o build/models.o build/track.o build/numerics.o"
while [ $# -ge 2 ]; do
  TAG=$1; DEFS=$2; shift 2
  $HIPCC $FLAGS $DEFS -c kin_ltv.hip -o build/kin_ltv_$TAG.o
  $HIPCC $FLAGS $DEFS -DVC_TIMING -c kin_ltv.hip -o build/kin_ltv_timing_$TAG.o
  $HIPCC -shared --offload-arch=gfx950 -o ../vcmpc/libvcmpc_$TAG.so build/kin_ltv_$TAG.o $OTHER
  $HIPCC -shared --offload-arch=gfx950 -o ../vcmpc/libvcmpc_timing_$TAG.so build/kin_ltv_timing_$TAG.o $OTHER_T
  echo "built $TAG ($DEFS)"
done
