"""Per-kernel means of rocprofv3 counter passes: for every kernel whose name
contains one of the --match substrings, the mean over its dispatches of
each counter collected in the given pass directories (one pass per
directory, `tools/gpu.sh pmcpy` steps), and the mean dispatch time where a
kernel trace rode along.  Prints one JSON object.

    python tools/pmc_by_kernel.py --match k_spmv_merged,k_pull_group gpurun_out/x/pmc3 gpurun_out/x/pmc4
"""
import argparse
import csv
import json
import os


def _csvs(d, suffix):
    for r, _, fs in os.walk(d):
        for f in fs:
            if f.endswith(suffix):
                yield os.path.join(r, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--match", default="k_spmv")
    a = ap.parse_args()
    keys = a.match.split(",")
    out = {}
    for d in a.dirs:
        per = {}
        for f in _csvs(d, "counter_collection.csv"):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if not any(k in name for k in keys):
                    continue
                k = (name, int(r["Dispatch_Id"]))
                per.setdefault(k, {}).setdefault(r["Counter_Name"], 0.0)
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                per[k]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        by_name = {}
        for (name, _), ctr in per.items():
            by_name.setdefault(name, []).append(ctr)
        for name, lst in by_name.items():
            o = out.setdefault(name, {"dispatches": len(lst)})
            for c in lst[0]:
                if c == "_ns":
                    o.setdefault("ns_under_counters", []).append(round(sum(x[c] for x in lst) / len(lst)))
                else:
                    o[c] = round(sum(x.get(c, 0.0) for x in lst) / len(lst), 1)
    print(json.dumps({"tool": "pmc_by_kernel", "passes": a.dirs, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
