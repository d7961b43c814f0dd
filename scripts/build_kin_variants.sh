#!/bin/bash
# A/B builds of one kernel source: libvcmpc_<tag>.so (and a timing build libvcmpc_timing_<tag>.so)
# with $SRC (default kin_ltv) compiled under extra -D flags, every other object shared with the
# default build.  Use them through VCMPC_LIB=...
# usage: [SRC=kin_ric] bash scripts/build_kin_variants.sh tag "-DFLAG=.." [tag "-D.." ...]
set -e
cd "$(dirname "$0")/../vehicle-control_amd/csrc"
make -j8 >/dev/null
make timing -j8 >/dev/null
HIPCC=/opt/rocm/bin/hipcc
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. -Wall -Wno-unused-function"
SRC=${SRC:-kin_ltv}
ALL="vcmpc_abi kin_ltv kin_ric kin_merit dyn_sqp casc_sqp casc_ric st_sqp models track numerics"
TIMED="vcmpc_abi kin_ltv kin_ric dyn_sqp casc_sqp casc_ric st_sqp"
case " $SRC " in " st_sqp "|" casc_ric "|" casc_sqp ") FLAGS="$FLAGS -mllvm -disable-machine-licm";; esac
OTHER=""; OTHER_T=""
for o in $ALL; do
  [ "$o" = "$SRC" ] && continue
  OTHER="$OTHER build/$o.o"
  if [[ " $TIMED " == *" $o "* ]]; then OTHER_T="$OTHER_T build/${o}_timing.o"; else OTHER_T="$OTHER_T build/$o.o"; fi
done
while [ $# -ge 2 ]; do
  TAG=$1; DEFS=$2; shift 2
  $HIPCC $FLAGS $DEFS -c $SRC.hip -o build/${SRC}_$TAG.o
  $HIPCC $FLAGS $DEFS -DVC_TIMING -c $SRC.hip -o build/${SRC}_timing_$TAG.o
  $HIPCC -shared --offload-arch=gfx950 -o ../vcmpc/libvcmpc_$TAG.so build/${SRC}_$TAG.o $OTHER
  $HIPCC -shared --offload-arch=gfx950 -o ../vcmpc/libvcmpc_timing_$TAG.so build/${SRC}_timing_$TAG.o $OTHER_T
  echo "built $TAG ($DEFS)"
done
