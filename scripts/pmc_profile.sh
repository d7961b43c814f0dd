#!/bin/bash
# PMC counter passes (one rocprofv3 run per pass, --pmc with --kernel-trace only)
# over a short bench run.  usage: bash scripts/pmc_profile.sh <tag> [batch]
set -u
TAG=${1:-r01}
B=${2:-1024}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for SET in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
           "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INST_LEVEL_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "== pass $i: $SET"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $SET -d "$OUT/p$i" -o run -f csv -- \
      python3 "$ROOT/bench.py" --steps 5 --warmup 1 --batch "$B" --no-cpu-baseline > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "   rc=$rc"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
done
find "$OUT" -name "*counter_collection*.csv" | head -20
