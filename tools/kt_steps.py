"""Per-step kernel time from a rocprofv3 kernel trace (--kernel-trace CSV).

A step starts at each launch of the kernel named --start (substring) and
runs to the next one; only kernels whose names contain one of --kernels (and
--filter, e.g. '<double') count.  Prints, as JSON: steps found, the median
sum of kernel durations per step, the median wall span per step (first start
to last end of the counted kernels), and per kernel name the median summed
duration per step.

    python tools/kt_steps.py TRACE.csv --start k_pack_group \
        --kernels k_pack_group,k_pull_group,k_spmv_sell_group,k_spmv_long --filter '<double' [--bytes B]
"""
import argparse
import csv
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--start", required=True)
    ap.add_argument("--kernels", required=True)
    ap.add_argument("--filter", default="")
    ap.add_argument("--bytes", type=float, default=0.0, help="bytes per step: adds GB/s of the kernel sum")
    ap.add_argument("--skip", type=int, default=0, help="steps to drop at the start (warmup)")
    a = ap.parse_args()
    path = a.trace
    if os.path.isdir(path):
        path = [os.path.join(r, f) for r, _, fs in os.walk(path) for f in fs if f.endswith("kernel_trace.csv")][0]
    names = a.kernels.split(",")
    ks = []
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        if a.filter and a.filter not in n:
            continue
        if any(s in n for s in names):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("(")[0]))
    ks.sort()
    steps, cur = [], None
    for k in ks:
        if a.start in k[2]:
            if cur:
                steps.append(cur)
            cur = [k]
        elif cur is not None:
            cur.append(k)
    if cur:
        steps.append(cur)
    steps = steps[a.skip:]
    if not steps:
        print(json.dumps({"error": "no steps"}))
        return
    med = lambda v: sorted(v)[len(v) // 2]
    sums = [sum(e - s for s, e, _ in st) for st in steps]
    spans = [max(e for _, e, _ in st) - min(s for s, _, _ in st) for st in steps]
    per = defaultdict(list)
    for st in steps:
        acc = defaultdict(int)
        for s, e, n in st:
            acc[n] += e - s
        for n, v in acc.items():
            per[n].append(v)
    out = {"trace": path, "steps": len(steps), "kernel_sum_us_median": med(sums) / 1e3,
           "span_us_median": med(spans) / 1e3,
           "per_kernel_us_median": {n: med(v) / 1e3 for n, v in per.items()}}
    if a.bytes:
        out["kernel_sum_gbs"] = a.bytes / (med(sums) * 1e-9) / 1e9
        out["span_gbs"] = a.bytes / (med(spans) * 1e-9) / 1e9
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
