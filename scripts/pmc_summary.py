"""Summarise the rocprofv3 PMC passes of scripts/pmc_profile.sh into one JSON per solve kernel:
counters averaged per dispatch (grouped by kernel template and grid size, i.e. per bench leg)
and the derived figures bench.py and DESIGN.md quote -- HBM traffic per launch (FETCH_SIZE +
WRITE_SIZE; FETCH_SIZE also doubled, the gfx950 correction for 16-B-per-lane streaming reads of
MI355X_MICROARCH.md, as an upper bracket), VALU / LDS instructions per wave, wait and LDS
bank-conflict fractions, and MFMA work (MOPS x 512 FLOPs) and busy cycles.

    python scripts/pmc_summary.py gpurun_out/pmc_r02 profiles/r02
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SOLVE_KERNELS = ("kin_ltv_kernel", "kin_ric_kernel", "dyn_sqp_kernel", "st_sqp_kernel", "casc_ric_kernel",
                 "casc_sqp_kernel")


def short_name(name):
    m = re.search(r"(\w+_kernel)<([^>]*)>", name)
    if not m:
        m2 = re.search(r"(\w+_kernel)I(.*?)E", name)
        return name[:60] if not m2 else m2.group(1)
    return f"{m.group(1)}<{m.group(2).replace(' ', '')}>"


def main():
    src = sys.argv[1]
    dst = sys.argv[2] if len(sys.argv) > 2 else None
    acc = defaultdict(lambda: defaultdict(list))   # (kernel, grid) -> counter -> values
    meta = {}
    for f in glob.glob(os.path.join(src, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row["Kernel_Name"]
                if not any(k in name for k in SOLVE_KERNELS):
                    continue
                key = (short_name(name), int(row["Grid_Size"]))
                acc[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
                meta[key] = dict(lds=int(row["LDS_Block_Size"]), scratch=int(row["Scratch_Size"]),
                                 vgpr=int(row["VGPR_Count"]), agpr=int(row["Accum_VGPR_Count"]),
                                 sgpr=int(row["SGPR_Count"]), workgroup=int(row["Workgroup_Size"]))
    out = {}
    for key, counters in sorted(acc.items()):
        kname, grid = key
        c = {k: sum(v) / len(v) for k, v in counters.items()}
        waves = c.get("SQ_WAVES") or grid / max(meta[key]["workgroup"], 1)
        d = {}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            d["fetch_bytes_per_launch"] = c["FETCH_SIZE"] * 1024
            d["write_bytes_per_launch"] = c["WRITE_SIZE"] * 1024
            d["traffic_bytes_per_launch"] = d["fetch_bytes_per_launch"] + d["write_bytes_per_launch"]
            d["traffic_bytes_per_launch_fetch_x2"] = 2 * d["fetch_bytes_per_launch"] + d["write_bytes_per_launch"]
        if "SQ_INSTS_VALU" in c:
            d["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / waves
        if "SQ_INSTS_LDS" in c:
            d["lds_insts_per_wave"] = c["SQ_INSTS_LDS"] / waves
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
            if "SQ_WAIT_ANY" in c:
                d["wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
            if "SQ_ACTIVE_INST_ANY" in c:
                d["active_inst_frac"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_ACTIVE_INST_LDS"):
            d["lds_bank_conflict_frac_of_lds_active"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"]
        for t in ("F64", "F32"):
            k = f"SQ_INSTS_VALU_MFMA_MOPS_{t}"
            if k in c:
                d[f"mfma_flops_{t.lower()}_per_launch"] = c[k] * 512
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            d["mfma_busy_cycles_per_launch"] = c["SQ_VALU_MFMA_BUSY_CYCLES"]
        out[f"{kname} grid={grid}"] = dict(kernel=kname, grid_threads=grid, resources=meta[key],
                                           dispatches=max(len(v) for v in counters.values()),
                                           counters_per_dispatch=c, derived=d)
    text = json.dumps(out, indent=1)
    print(text)
    if dst:
        os.makedirs(dst, exist_ok=True)
        with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
