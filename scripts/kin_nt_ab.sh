#!/bin/bash
# A/B of kin_ltv's output stores (KIN_NT_OUT): C2 bench leg time and a FETCH_SIZE / WRITE_SIZE pass
# each, default library vs libvcmpc_nt.so.  usage: bash scripts/kin_nt_ab.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ntab_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
LEGS="--no-c3 --no-c4 --no-c5 --no-casc --no-kin-legs --no-latency --no-cpu-baseline"
for v in default nt; do
  unset VCMPC_LIB
  [ "$v" != default ] && export VCMPC_LIB="$ROOT/vehicle-control_amd/vcmpc/libvcmpc_$v.so"
  (cd "$ROOT" && timeout -k 10 300 python bench.py $LEGS > "$OUT/bench_$v.log" 2>&1) || exit $?
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d "$OUT/${v}_$c" -o run -f csv -- \
        python3 "$ROOT/bench.py" --steps 3 --warmup 1 $LEGS > "$OUT/${v}_$c.log" 2>&1) || exit $?
  done
done
cd "$ROOT"
python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
for v in ("default", "nt"):
    d = json.loads([l for l in open(f"{out}/bench_{v}.log") if l.startswith("{")][-1])
    row = [v, round(d["value"]), round(d["roofline"]["kernel_ms"], 4)]
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"{out}/{v}_{c}/**/*counter_collection.csv", recursive=True)[0]
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
                if "kin_ltv_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c and r["Grid_Size"] == "65536"]
        row.append(f"{c} {sum(vals) / len(vals) * 1024 / 1e6:.3f} MB")
    print(row)
PY
