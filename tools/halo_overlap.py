"""Halo / interior overlap on one GPU, read from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o ov -- \
        python tools/halo_overlap.py run [--n 128] [--shape 2,2,2] [--steps 20]
    python tools/halo_overlap.py analyze DIR/.../ov_kernel_trace.csv

`run`: the (2,2,2) weak-scaling partition (n^3 nodes per part) with all parts
in this process on device 0, mul! repeated `steps` times.  The parts share
one stream pair, so each mul! is: pack (all parts, compute stream) → pull-
unpack (all parts, comm stream) ‖ interior slices (all parts, compute
stream) → boundary slices.  `analyze`: per mul!, the interval of the pull
kernel and of the interior SpMV kernel(s) launched after the same pack, and
how much of the pull ran while an interior kernel was running."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(argv):
    import argparse
    import numpy as np
    sys.path.insert(0, ROOT)
    import pamd
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--shape", default="2,2,2")
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args(argv)
    shape = tuple(int(v) for v in a.shape.split(","))
    be = pamd.HIPBackend(devices=[0])
    parts = be.get_part_ids(shape)
    N = tuple(a.n * s for s in shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    for _ in range(a.steps):
        pamd.mul_(y, A, x)
    be.context(1).sync()


def analyze(path):
    if os.path.isdir(path):  # a rocprofv3 -d directory: its kernel trace
        found = [os.path.join(r, f) for r, _, fs in os.walk(path) for f in fs if f.endswith("kernel_trace.csv")]
        if not found:
            print(json.dumps({"error": f"no kernel_trace.csv under {path}"}))
            return
        path = found[0]
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows),
                key=lambda t: t[0])
    steps = []
    i = 0
    while i < len(ks):
        if "k_pack_group" not in ks[i][2]:
            i += 1
            continue
        pack = ks[i]
        j = i + 1
        pull, interior = None, []
        while j < len(ks) and "k_pack_group" not in ks[j][2]:
            k = ks[j]
            if "k_pull_group" in k[2] and pull is None:
                pull = k
            elif "k_spmv_sell_group" in k[2] and (pull is None or k[0] < pull[1]):
                interior.append(k)
            j += 1
        if pull is not None and interior:
            lo = max(pull[0], min(k[0] for k in interior))
            hi = min(pull[1], max(k[1] for k in interior))
            steps.append({"pack_us": (pack[1] - pack[0]) / 1e3, "pull_us": (pull[1] - pull[0]) / 1e3,
                          "interior_us": (max(k[1] for k in interior) - min(k[0] for k in interior)) / 1e3,
                          "pull_hidden_frac": max(0, hi - lo) / max(1, pull[1] - pull[0]),
                          "pull_start_after_interior_start_us": (pull[0] - min(k[0] for k in interior)) / 1e3})
        i = j
    if not steps:
        print(json.dumps({"error": "no pack → pull ‖ interior sequence found"}))
        return
    med = lambda key: sorted(s[key] for s in steps)[len(steps) // 2]
    print(json.dumps({"steps": len(steps), "median": {k: round(med(k), 3) for k in steps[0]},
                      "min_hidden_frac": round(min(s["pull_hidden_frac"] for s in steps), 3),
                      "per_step": steps}, indent=1))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "run":
        run(sys.argv[2:])
    elif len(sys.argv) > 2 and sys.argv[1] == "analyze":
        analyze(sys.argv[2])
    else:
        print(__doc__)
        sys.exit(2)
