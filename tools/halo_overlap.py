"""Halo / interior overlap on one GPU, read from a rocprofv3 kernel trace.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o ov -- \
        python tools/halo_overlap.py run [--n 128] [--shape 2,2,2] [--steps 20]
    python tools/halo_overlap.py analyze DIR/.../ov_kernel_trace.csv

`run`: the (2,2,2) weak-scaling partition (n^3 nodes per part) with all parts
in this process on device 0, mul! repeated `steps` times.
  --mode pull: the parts share one stream pair and the grouped mul! packs
    (compute stream), pulls (comm stream) ‖ interior slices, then boundary
    slices (pa_tune halo_direct = 0; the default direct pull has no transport
    to overlap);
  --mode rccl: the multi-GPU path — per part: pack, the halo as one RCCL
    group of ncclSend/ncclRecv on the comm stream (here to self, one GPU)
    ‖ interior slices, then unpack and the boundary slices.
`analyze`: per mul!, the interval of the transport kernel(s) (pull or RCCL)
and of the interior SpMV kernels launched after the packs, and how much of
the transport ran while an interior kernel was running."""
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
    ap.add_argument("--mode", default="pull", choices=["pull", "rccl"])
    a = ap.parse_args(argv)
    shape = tuple(int(v) for v in a.shape.split(","))
    if a.mode == "pull":
        pamd._lib.tune("halo_direct", 0)
    be = pamd.HIPBackend(devices=[0], rccl=a.mode == "rccl")
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
    is_pack = lambda n: "k_pack" in n
    is_xport = lambda n: "k_pull_group" in n or "nccl" in n.lower()
    is_spmv = lambda n: "k_spmv" in n
    i = 0
    while i < len(ks):
        if not is_pack(ks[i][2]):
            i += 1
            continue
        j = i
        packs = []
        while j < len(ks) and is_pack(ks[j][2]):
            packs.append(ks[j])
            j += 1
        xport, interior = [], []
        while j < len(ks) and not is_pack(ks[j][2]):
            k = ks[j]
            if is_xport(k[2]):
                xport.append(k)
            elif is_spmv(k[2]):
                interior.append(k)
            j += 1
        if xport and interior:
            t0, t1 = min(k[0] for k in xport), max(k[1] for k in xport)
            interior = [k for k in interior if k[0] < t1]  # launched before the transport ended
        if xport and interior:
            lo = max(t0, min(k[0] for k in interior))
            hi = min(t1, max(k[1] for k in interior))
            steps.append({"pack_us": (packs[-1][1] - packs[0][0]) / 1e3, "pull_us": (t1 - t0) / 1e3,
                          "interior_us": (max(k[1] for k in interior) - min(k[0] for k in interior)) / 1e3,
                          "pull_hidden_frac": max(0, hi - lo) / max(1, t1 - t0),
                          "pull_start_after_interior_start_us": (t0 - min(k[0] for k in interior)) / 1e3,
                          "transport": "rccl" if any("nccl" in k[2].lower() for k in xport) else "pull"})
        i = j
    if not steps:
        print(json.dumps({"error": "no pack → pull ‖ interior sequence found"}))
        return
    med = lambda key: sorted(s[key] for s in steps)[len(steps) // 2]
    num = [k for k in steps[0] if k != "transport"]
    print(json.dumps({"steps": len(steps), "transport": steps[0]["transport"],
                      "median": {k: round(med(k), 3) for k in num},
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
