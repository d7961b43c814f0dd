#!/bin/bash
# PMC counter passes, one rocprofv3 run per pass (--pmc with --kernel-trace only, no trace
# domains), over a short bench run of every solve leg except the C5 closed loop (1,500
# dispatches) and the converged-setting legs (--no-converged: they launch the same st_sqp<60> /
# casc_ric kernels on the same grid at 40 SQP iterations, and a per-dispatch average over both
# settings -- the round-5 summary's -- mixed 5- and 40-iteration launches).  Counters the box does not list are dropped from a pass before it runs, and
# every pass is held to the per-block limits (<= 8 SQ, <= 4 TCC: FETCH_SIZE and WRITE_SIZE
# get passes of their own).  Summaries: python scripts/pmc_summary.py gpurun_out/pmc_<tag>
# usage: bash scripts/pmc_profile.sh <tag> [extra bench args]
set -u
TAG=${1:-r02}
shift || true
EXTRA="$*"
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
have() { grep -qw "$1" "$OUT/counters_list.txt"; }
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  KEEP=""
  for c in $SET; do if have "$c"; then KEEP="$KEEP $c"; else echo "   (counter $c not listed, dropped)"; fi; done
  [ -z "$KEEP" ] && continue
  echo "== pass $i:$KEEP"
  timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --pmc $KEEP -d "$OUT/p$i" -o run -f csv -- \
      python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-c5 --no-cpu-baseline --no-latency --no-converged $EXTRA > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "   rc=$rc"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
done
find "$OUT" -name "*counter_collection*.csv" | head -20
