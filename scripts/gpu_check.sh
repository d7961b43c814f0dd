#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fatal exit (timeout/abort/segfault,
# rc >= 124) ends the script so nothing else touches a sick GPU.
# usage: bash scripts/gpu_check.sh [tag] [steps]
set -u
TAG=${1:-r01}
STEPS=${2:-20}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <log> <timeout> cmd...
  local log=$1 lim=$2; shift 2
  echo "== $* (limit ${lim}s) -> $log"
  timeout -k 10 "$lim" "$@" > "$OUT/$log" 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -n 5 "$OUT/$log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc, stopping"; exit $rc; fi
  return 0
}
cd "$ROOT"
run pytest_gpu_$TAG.log 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
run smoke_$TAG.log 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_$TAG.log 600 python bench.py --steps "$STEPS" --warmup 3
cd /tmp
run rocprof_$TAG.log 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps "$STEPS" --warmup 3 --no-cpu-baseline
find "$OUT/prof_$TAG" -name "*stats*" | head
