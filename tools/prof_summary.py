"""Summarise a scripts/profile.sh output directory: per-kernel launch groups
(split by grid size, so the pattern-slice, side-SELL and int32-reference
SpMV launches are separate lines) and the PMC passes per SpMV launch.
Usage: python tools/prof_summary.py gpurun_out/prof > profiles/.../summary.txt"""
import csv
import os
import sys
from collections import defaultdict


def trace_groups(path):
    g = defaultdict(list)
    for r in csv.DictReader(open(path)):
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        g[(r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]))].append(d)
    return g


def pmc(path):
    agg = defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[(r["Kernel_Name"].split("(")[0], int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0),
             r["Counter_Name"])].append(float(r["Counter_Value"]))
    return agg


def main(d):
    for sub in ("kt", "cg"):
        p = os.path.join(d, sub, f"{sub}_kernel_trace.csv")
        if not os.path.exists(p):
            continue
        print(f"== {sub}: kernel launches grouped by (kernel, grid threads), durations in us")
        g = trace_groups(p)
        for (k, grid), v in sorted(g.items(), key=lambda kv: -sum(kv[1])):
            v = sorted(v)
            print(f"{k[:60]:60s} grid {grid:>10d}  calls {len(v):4d}  avg {sum(v) / len(v) / 1e3:9.2f}"
                  f"  median {v[len(v) // 2] / 1e3:9.2f}  min {v[0] / 1e3:9.2f}")
    for sub, fn in (("fetch", "fetch"), ("write", "write"), ("sq", "sq")):
        p = os.path.join(d, sub, f"{fn}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        print(f"== pmc pass {sub}: mean per launch (SpMV kernels)")
        for (k, grid, c), v in sorted(pmc(p).items()):
            if "spmv" in k:
                print(f"{k[:45]:45s} grid {grid:>10d} {c:18s} n={len(v):3d} mean {sum(v) / len(v):.6g}")


if __name__ == "__main__":
    main(sys.argv[1])
