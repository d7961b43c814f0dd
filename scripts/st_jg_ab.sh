#!/bin/bash
# A/B of the single-track kernel's stage-Jacobian placement (round 5): the default library
# (J in a global workspace for N >= 45: four workgroups per CU) against variants built by
# SRC=st_sqp bash scripts/build_kin_variants.sh <tag> "<-D flags>" (jl: -DST_J_GLOBAL=0, J in LDS;
# jg3: J global but the block padded back to three workgroups per CU, -DST_LDS_PAD=23520).
# Bench legs C3 (N = 40) and single-track N = 60 (5 and 40 SQP iterations); LAT=1 adds the
# single-vehicle latency legs; CASC=0 drops the cascaded legs.
# usage: [LAT=1] [CASC=0] bash scripts/st_jg_ab.sh <tag> [variant ...]
TAG=$1; shift
VARS=${*:-default jl}
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
EXTRA="--no-latency"
[ -n "$LAT" ] && EXTRA="--latency-calls 50"
for v in $VARS; do
  lib=""
  [ "$v" != default ] && lib="VCMPC_LIB=$(pwd)/vehicle-control_amd/vcmpc/libvcmpc_$v.so"
  env $lib timeout -k 10 300 python -u bench.py --no-c4 --no-c5 ${CASC:+--no-casc} --no-kin-legs --no-cpu-baseline \
    $EXTRA > "$OUT/stjg_${TAG}_$v.log" 2>&1 || exit $?
  echo "$v done"
done
