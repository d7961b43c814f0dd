#!/bin/bash
# One PMC pass (wave cycles, busy cycles, GUI-active cycles) + kernel trace over the C3 / N = 60
# bench legs for each library variant: per-wave duration and clock under each occupancy
# (st_jg_ab.sh's variants).  usage: bash scripts/st_occ_pmc.sh <tag> [variant ...]
TAG=$1; shift
VARS=${*:-default jl}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/occ_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for v in $VARS; do
  unset VCMPC_LIB
  [ "$v" != default ] && export VCMPC_LIB="$ROOT/vehicle-control_amd/vcmpc/libvcmpc_$v.so"
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
      SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$OUT/$v" -o run -f csv -- \
      python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-c4 --no-c5 --no-casc --no-kin-legs --no-cpu-baseline \
      --no-latency > "$OUT/$v.log" 2>&1
  rc=$?
  echo "$v rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
