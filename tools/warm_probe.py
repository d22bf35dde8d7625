"""Does the headline operator's SpMV time drift over the first seconds of
sustained load (clock / power ramp), independently of which operator copy
runs?  Builds K copies of the one-part FE27 n³ operator, then times spans
of R back-to-back mul! calls, cycling over the copies for several rounds,
and prints every span's ms per mul! with its copy and the elapsed time.

    python tools/warm_probe.py [--n 256] [--k 2] [--rounds 12] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--k", type=int, default=2)
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--torch", action="store_true", help="initialise torch's HIP context first (as bench.py does)")
a = ap.parse_args()
if a.torch:
    import torch
    torch.zeros(1, device="cuda")
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
ctx = be.context(1)
N = (a.n,) * 3
partition = pamd.drivers.stencil_partition(parts, N, 27)
As = [pamd.drivers.stencil_operator(parts, N, 27, np.float64, partition=partition) for _ in range(a.k)]
x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids),
                                          As[0].cols.partition), As[0].cols)
ys = [pamd.PVector.undef(A.rows) for A in As]
ctx.sync()
t0 = time.perf_counter()
spans = []
for rnd in range(a.rounds):
    for i, A in enumerate(As):
        ctx.span_start()
        for _ in range(a.reps):
            pamd.mul_(ys[i], A, x)
        ctx.span_stop()
        ms = ctx.span_ms() / a.reps
        spans.append({"round": rnd, "copy": i, "ms": round(ms, 4), "t_s": round(time.perf_counter() - t0, 3)})
print(json.dumps({"tool": "warm_probe", "n": a.n, "k": a.k, "reps": a.reps, "spans": spans}))
