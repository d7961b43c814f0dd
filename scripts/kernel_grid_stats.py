"""Per-(kernel, grid size) dispatch statistics from a rocprofv3 kernel trace: the bench process
launches kin_ltv_kernel<20> at two grid sizes (C2's B = 1024 and C4's shard), which
rocprofv3 --stats averages together; this splits them so the C2 launch's average can be set
beside bench.py's live HIP-event figure.

    python scripts/kernel_grid_stats.py gpurun_out/prof_<tag>/run_kernel_trace.csv > profiles/<r>/kernel_grid_stats_<tag>.csv
"""
import collections
import csv
import sys


def main(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["LDS_Block_Size"]), int(r["Scratch_Size"]),
             int(r["VGPR_Count"]))].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "GridX", "Problems", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Calls", "AverageNs",
                "MinNs", "MaxNs"])
    for (n, g, lds, scr, vg), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        if "rocclr" in n or "at::native" in n:
            continue
        w.writerow([n, g, g // 64, lds, scr, vg, len(v), round(sum(v) / len(v), 1), min(v), max(v)])


if __name__ == "__main__":
    main(sys.argv[1])
