"""Is the headline's time a property of the operator or of when it runs?
In one process: the one-part 256³ FE27 operator (the headline) and the same
operator on (2,2,2) parts of the GPU (bench.py's halo_1gpu), timed in
alternation, K mul! each, several rounds, after a short and then after a
long warm phase; the GPU's clocks (rocm-smi, read only) before and after.

    python tools/order_probe.py [--n 256] [--k 20] [--rounds 4]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402


def clocks():
    try:
        out = subprocess.run(["rocm-smi", "--showclocks"], capture_output=True, text=True, timeout=30).stdout
        return [l.strip() for l in out.splitlines() if "clk" in l.lower()][:8]
    except Exception as e:  # noqa: BLE001
        return [repr(e)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    be = pamd.HIPBackend(devices=[0])
    probs = {}
    for shape in ((1, 1, 1), (2, 2, 2)):
        parts = be.get_part_ids(shape)
        A = pamd.drivers.stencil_operator(parts, (a.n,) * 3, 27)
        x = pamd.PVector.from_host(pamd.map_parts(
            lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
        y = pamd.PVector.undef(A.rows)
        probs[shape] = (A, x, y, [be.context(p, len(parts.part_ids)) for p in parts.part_ids])
    c_before = clocks()

    def run(shape, k):
        A, x, y, ctxs = probs[shape]
        for c in ctxs:
            c.sync()
        t0 = time.perf_counter()
        for _ in range(k):
            pamd.mul_(y, A, x)
        for c in ctxs:
            c.sync()
        return 1e3 * (time.perf_counter() - t0) / k

    seq = []
    for shape in ((1, 1, 1), (2, 2, 2)):  # cold: 2 untimed calls only
        run(shape, 2)
    for r in range(a.rounds):
        for shape in ((1, 1, 1), (2, 2, 2)):
            seq.append({"phase": "short warm", "round": r, "shape": list(shape), "ms": round(run(shape, a.k), 4)})
    # a long warm phase: ~2 s of mul! on the headline operator
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        run((1, 1, 1), 20)
    c_mid = clocks()
    for r in range(a.rounds):
        for shape in ((1, 1, 1), (2, 2, 2)):
            seq.append({"phase": "after 2 s warm", "round": r, "shape": list(shape), "ms": round(run(shape, a.k), 4)})
    # idle 3 s, then again
    time.sleep(3.0)
    for shape in ((1, 1, 1), (2, 2, 2)):
        seq.append({"phase": "after 3 s idle", "round": 0, "shape": list(shape), "ms": round(run(shape, a.k), 4)})
    print(json.dumps({"tool": "order_probe", "n": a.n, "k": a.k, "clocks_before": c_before, "clocks_after_warm": c_mid,
                      "clocks_end": clocks(), "sequence": seq}, indent=1))


if __name__ == "__main__":
    main()
