"""A/B the SpMV kernel variants (pa_tune knobs) in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24).  Kernel time from HIP events
on the SpMV's stream.  Usage: python tools/ab_spmv.py [--n 256] [--rounds 5]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--kind", type=int, default=27)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--variants", default="2:4,3:4,0:4,1:4,2:8,3:8")
a = ap.parse_args()

be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
N = (a.n,) * 3
A = pamd.drivers.stencil_operator(parts, N, a.kind)
x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(1).uniform(-1, 1, s.num_lids),
                                          A.cols.partition), A.cols)
y = pamd.PVector.undef(A.rows)
ctx = be.context(1)
info = A.values.local(1).info()
B = info["nnz"] * 12 + (info["nrows"] + 1) * 4 + info["nrows"] * 16
variants = [tuple(int(t) for t in v.split(":")) for v in a.variants.split(",")]
res = {v: [] for v in variants}
ref = None
for rnd in range(a.rounds):
    for v in variants:
        pamd._lib.tune("spmv_flags", v[0])
        pamd._lib.tune("spmv_unroll", v[1])
        pamd.mul_(y, A, x)
        ctx.set_timing(True)
        for _ in range(a.reps):
            pamd.mul_(y, A, x)
            ms = sum(ctx.last_kernel_ms())
            res[v].append(ms)
        ctx.set_timing(False)
        out = y.to_host().local(1)
        if ref is None:
            ref = out
        assert np.array_equal(out, ref), f"variant {v} changed the result"
print(f"n={a.n} kind={a.kind} nnz={info['nnz']} bytes={B}")
for v in variants:
    t = np.array(res[v])
    print(f"flags={v[0]} unroll={v[1]}: median {np.median(t):.4f} ms  min {t.min():.4f}  "
          f"-> {B / np.median(t) / 1e6:.0f} GB/s (median), {B / t.min() / 1e6:.0f} (best)")
