"""Shrink one rocprofv3 output directory in place (gpu.sh runs it after each
profiled step, so a call's gpurun_out/ stays under gpurun's 64 MiB merge
cap): counter and kernel-trace rows are kept only for kernels whose name
matches PA_PROF_KEEP (a regex; default the SpMV, halo and probe kernels),
the per-kernel stats files are kept whole, other large CSVs are dropped.

    python tools/prune_prof.py DIR
"""
import csv
import os
import re
import sys

KEEP = re.compile(os.environ.get("PA_PROF_KEEP", r"k_spmv|k_pull|k_pack|k_unpack|k_probe|k_cg_|k_reduce"))


def prune(d):
    for r, _, fs in os.walk(d):
        for f in fs:
            p = os.path.join(r, f)
            if f.endswith(("kernel_stats.csv", "domain_stats.csv")):
                continue
            if f.endswith(("counter_collection.csv", "kernel_trace.csv")):
                rows = list(csv.reader(open(p)))
                if not rows:
                    continue
                head, body = rows[0], rows[1:]
                k = head.index("Kernel_Name") if "Kernel_Name" in head else None
                keep = [row for row in body if k is None or KEEP.search(row[k])]
                with open(p, "w", newline="") as fh:
                    w = csv.writer(fh)
                    w.writerow(head)
                    w.writerows(keep)
            elif os.path.getsize(p) > (1 << 20):
                os.remove(p)


if __name__ == "__main__":
    for d in sys.argv[1:]:
        if os.path.isdir(d):
            prune(d)
