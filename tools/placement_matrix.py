"""Which buffer's placement moves the SpMV time: the matrix's or the
vectors'?  K copies of the FE27 operator (one part) and K (x, y) pairs,
built one after the other; every (A_i, x_j, y_j) combination timed in
interleaved rounds (HIP events on the part's stream).  Prints one JSON
object with the K x K table of ms per mul! and the vectors' addresses.

    python tools/placement_matrix.py [--n 256] [--k 3] [--rounds 4] [--reps 20]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--shape", default="1,1,1")
    ap.add_argument("--tune", default="", help="pa_tune knobs before anything is built: key=v[,key=v]")
    a = ap.parse_args()
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        pamd._lib.tune(k, int(v))
    be = pamd.HIPBackend(devices=[0])
    shape = tuple(int(v) for v in a.shape.split(","))
    parts = be.get_part_ids(shape)
    N = tuple(a.n * s for s in shape)
    partition = pamd.drivers.stencil_partition(parts, N, 27)
    ctx = be.context(parts.part_ids[0])
    As, xs, ys = [], [], []
    for k in range(a.k):
        As.append(pamd.drivers.stencil_operator(parts, N, 27, np.float64, partition=partition))
    for k in range(a.k):
        A = As[0]
        xs.append(pamd.PVector.from_host(pamd.map_parts(
            lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols))
        ys.append(pamd.PVector.undef(A.rows))
    ctx.sync()
    t = {(i, j): [] for i in range(a.k) for j in range(a.k)}
    ref = None
    for _ in range(a.rounds):
        for i in range(a.k):
            for j in range(a.k):
                # A_i was built on its own copy of the ranges: x/y must share A_i's layout
                x = xs[j]
                y = ys[j]
                pamd.mul_(y, As[i], x)
                ctx.sync()
                ctx.span_start()
                for _ in range(a.reps):
                    pamd.mul_(y, As[i], x)
                ctx.span_stop()
                t[(i, j)].append(ctx.span_ms() / a.reps)
                if ref is None:
                    ref = y.to_host().parts[0].copy()
    table = [[round(float(np.median(t[(i, j)])), 4) for j in range(a.k)] for i in range(a.k)]
    print(json.dumps({"tool": "placement_matrix", "tune": a.tune, "n": a.n, "shape": a.shape, "k": a.k,
                      "ms_A_rows_x_cols": table,
                      "x_va": [hex(v.values.parts[0].device_ptr()) for v in xs],
                      "y_va": [hex(v.values.parts[0].device_ptr()) for v in ys]}))


if __name__ == "__main__":
    main()
