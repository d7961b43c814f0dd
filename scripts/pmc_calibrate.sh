#!/bin/bash
# FETCH_SIZE and WRITE_SIZE (one rocprofv3 pass each: FETCH_SIZE takes 3 of the 4 TCC counters)
# over scripts/pmc_calibrate.py's known byte counts.  usage: bash scripts/pmc_calibrate.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmccal_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$c" -o run -f csv -- \
      python3 "$ROOT/scripts/pmc_calibrate.py" > "$OUT/$c.log" 2>&1 || exit $?
done
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
n = 1 << 24
for c, ref in (("FETCH_SIZE", 8 * n), ("WRITE_SIZE", 32 * n)):
    f = glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True)[0]
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "rcp_probe" in r["Kernel_Name"] and r["Counter_Name"] == c]
    print(f"{c}: {len(v)} launches, per launch {[round(x) for x in v]} (KB units) -> {[round(x * 1024 / ref, 3) for x in v]} of the {ref} B the kernel moves")
PY
