"""Per-leg kernel statistics from one rocprofv3 pass over bench.py.

bench.py wraps each timed leg in a roctx range "leg:<name>" (leg_push / leg_pop).  The same
kernel runs in several legs: kin_ltv_kernel<20> in C2 and C4, st_sqp_kernel<60> at 5 and at 40
SQP iterations, casc_ric at 3 and 40.  A per-kernel or per-grid average therefore mixes legs.
This script assigns every dispatch of the kernel trace to the leg range that contains it (start
and end inside the range's host timestamps, same clock in rocprofv3's traces) and prints one row
per (leg, kernel).  bench.py's `kernel_ms` of a leg is the mean HIP-event time of its timed
launches and must match the AverageNs of its row.

    rocprofv3 --kernel-trace --marker-trace --stats -f csv -d gpurun_out/prof_<tag> -o run -- python3 bench.py ...
    python scripts/leg_stats.py gpurun_out/prof_<tag> > profiles/<round>/kernel_leg_stats_<tag>.csv
"""
import collections
import csv
import glob
import os
import sys


def find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def marker_ranges(path):
    """[(leg, start, end)] from the marker API trace (roctxRangePushA / Pop pairs)."""
    rows = list(csv.DictReader(open(path)))
    out = []
    for r in rows:
        msg = r.get("Message") or r.get("Marker_Message") or r.get("Function") or ""
        if "leg:" not in msg:
            continue
        leg = msg[msg.index("leg:") + 4:].strip()
        out.append((leg, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return out


def main(d):
    legs = marker_ranges(find(d, "marker_api_trace.csv"))
    agg = collections.defaultdict(list)
    meta = {}
    for r in csv.DictReader(open(find(d, "kernel_trace.csv"))):
        n = r["Kernel_Name"]
        if "rocclr" in n or "at::native" in n or "elementwise" in n:
            continue
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        for leg, a, b in legs:
            if a <= t0 and t1 <= b:
                key = (leg, n, int(r["Grid_Size_X"]))
                agg[key].append(t1 - t0)
                meta[key] = (int(r["LDS_Block_Size"]), int(r["Scratch_Size"]), int(r["VGPR_Count"]))
                break
    w = csv.writer(sys.stdout)
    w.writerow(["Leg", "Name", "GridX", "Problems", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Calls",
                "AverageNs", "MinNs", "MaxNs"])
    order = {leg: i for i, (leg, _, _) in enumerate(legs)}
    for (leg, n, g), v in sorted(agg.items(), key=lambda kv: (order.get(kv[0][0], 99), -sum(kv[1]))):
        lds, scr, vg = meta[(leg, n, g)]
        w.writerow([leg, n, g, g // 64, lds, scr, vg, len(v), round(sum(v) / len(v), 1), min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
