#!/bin/bash
# Round-end measurement: the bench line, a rocprofv3 kernel-trace + marker-trace pass over every
# leg (bench.py wraps each timed leg in a roctx range; scripts/leg_stats.py splits the dispatches
# per leg, so C2 and C4 -- both kin_ltv_kernel<20> -- and the 3- and 40-iteration SQP legs get
# rows of their own), and the PMC passes (scripts/pmc_profile.sh).
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
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -f csv -d "$OUT/prof_$TAG" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-latency > "$OUT/rocprof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ge 124 ] && exit $rc
cd "$ROOT"
python scripts/leg_stats.py "$OUT/prof_$TAG" > "$OUT/kernel_leg_stats_$TAG.csv"
bash scripts/pmc_profile.sh "$TAG" --no-c4
