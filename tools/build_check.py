"""Are K operators built one after the other in one process the same
operator?  Builds K copies of the one-part FE27 n³ operator (device
generator, pa_mat_stencil), prints each copy's encoding (slice kinds, side
rows, bytes), the bitwise agreement of its mul! with copy 0's on one x, and
its kernel time (HIP events).  PA_HIP_LIB selects another build of the
library (A/B of library versions).

    python tools/build_check.py [--n 256] [--k 3] [--dtype f64]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--k", type=int, default=3)
ap.add_argument("--kind", type=int, default=27)
ap.add_argument("--dtype", default="f64")
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dtype = {"f64": np.float64, "f32": np.float32}[a.dtype]
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
ctx = be.context(1)
N = (a.n,) * 3
partition = pamd.drivers.stencil_partition(parts, N, a.kind)
As = [pamd.drivers.stencil_operator(parts, N, a.kind, dtype, partition=partition) for _ in range(a.k)]
x = pamd.PVector.from_host(pamd.map_parts(
    lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids).astype(dtype), As[0].cols.partition),
    As[0].cols)
ys = []
out = []
for i, A in enumerate(As):
    y = pamd.PVector.undef(A.rows, dtype)
    pamd.mul_(y, A, x)
    ctx.sync()
    ctx.span_start()
    for _ in range(a.reps):
        pamd.mul_(y, A, x)
    ctx.span_stop()
    ms = ctx.span_ms() / a.reps
    h = y.to_host().local(1)
    ys.append(h)
    f = A.values.local(1).info()
    out.append({"copy": i, "ms": round(ms, 4), "same_as_copy0": bool(np.array_equal(h.view(np.uint8), ys[0].view(np.uint8))),
                "y_sum": float(np.sum(h)), **{k: f[k] for k in ("nslices", "pattern_slices", "delta16_slices",
                                                                  "regular_rows", "side_rows", "value_bytes",
                                                                  "index_bytes", "meta_bytes", "slots", "nnz")}})
print(json.dumps({"tool": "build_check", "lib": pamd._lib.LIB_PATH, "n": a.n, "kind": a.kind, "dtype": a.dtype,
                  "copies": out}))
