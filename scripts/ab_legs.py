"""Print the throughput / kernel-time / latency fields of bench.py JSON lines side by side.
    python scripts/ab_legs.py gpurun_out/stjg_<tag>_*.log"""
import json
import sys


def fields(o, p=""):
    if isinstance(o, dict):
        for k, v in o.items():
            yield from fields(v, f"{p}.{k}" if p else k)
    elif isinstance(o, (int, float)) and not p.startswith("cpu") and any(
            t in p for t in ("value", "kernel_ms", "median_ms")) and "recorded" not in p:
        yield p, o


cols = {}
for path in sys.argv[1:]:
    with open(path) as f:
        line = [ln for ln in f if ln.startswith("{")][-1]
    cols[path.rsplit("_", 1)[-1].replace(".log", "")] = dict(fields(json.loads(line)))
keys = list(dict.fromkeys(k for c in cols.values() for k in c))
print(f"{'field':44s}" + "".join(f"{n:>14s}" for n in cols))
for k in keys:
    print(f"{k:44s}" + "".join(f"{c.get(k, float('nan')):14.6g}" for c in cols.values()))
