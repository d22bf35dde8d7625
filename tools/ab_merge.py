"""Interleaved A/B in one process: FE27 256^3 (one part) mul! with the merged
launch (pa_tune spmv_merge = 1) vs one launch per slice kind (0), HIP-event
span over --reps calls, --rounds rounds; every variant must give the same bits.
    python tools/ab_merge.py [--dtype f64] [--rounds 5] [--reps 20]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dtype", default="f64")
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--kind", type=int, default=27)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
dt = {"f64": np.float64, "f32": np.float32, "c128": np.complex128, "c64": np.complex64}[a.dtype]
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
A = pamd.drivers.stencil_operator(parts, (a.n,) * 3, a.kind, dt)
x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(1).uniform(-1, 1, s.num_lids).astype(dt),
                                          A.cols.partition), A.cols)
y = pamd.PVector.undef(A.rows, dt)
ctx = be.context(1)
res, ref = {0: [], 1: []}, None
for r in range(a.rounds):
    for m in (1, 0):
        pamd._lib.tune("spmv_merge", m)
        for _ in range(3):
            pamd.mul_(y, A, x)
        ctx.sync()
        ctx.span_start()
        for _ in range(a.reps):
            pamd.mul_(y, A, x)
        ctx.span_stop()
        res[m].append(ctx.span_ms() / a.reps)
        out = y.to_host().local(1)
        if ref is None:
            ref = out
        assert np.array_equal(out, ref)
pamd._lib.tune("spmv_merge", 1)
print(json.dumps({"dtype": a.dtype, "n": a.n, "kind": a.kind,
                  "merged_ms": [round(v, 4) for v in res[1]], "per_kind_ms": [round(v, 4) for v in res[0]],
                  "merged_median": round(float(np.median(res[1])), 4),
                  "per_kind_median": round(float(np.median(res[0])), 4)}))
