#!/bin/bash
# Round-end measurement: the bench line, a rocprofv3 kernel-stats pass over the headline legs
# without the C4 leg (C4 launches the same kin_ltv_kernel<20> on 65,536 problems, which would
# mix into the C2 kernel's average), and the PMC passes (scripts/pmc_profile.sh).
# usage: bash scripts/final_profile.sh <tag>
set -u
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > "$OUT/bench_$TAG.log" 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ge 124 ] && exit $rc
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-c4 > "$OUT/rocprof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ge 124 ] && exit $rc
cd "$ROOT"
bash scripts/pmc_profile.sh "$TAG" --no-c4
