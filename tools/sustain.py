"""Is the box's SpMV rate time-varying?  FE27 256^3 F64 mul! run back to back
for --seconds, the mean per-call time of each --window printed as JSON lines
(HIP-event span on the compute stream), plus the HBM probe every --probe-every
windows.  usage: python tools/sustain.py [--seconds 30] [--window 1.0]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seconds", type=float, default=30.0)
ap.add_argument("--window", type=float, default=1.0)
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--probe-every", type=int, default=5)
a = ap.parse_args()
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
A = pamd.drivers.stencil_operator(parts, (a.n,) * 3, 27)
x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(1).uniform(-1, 1, s.num_lids),
                                          A.cols.partition), A.cols)
y = pamd.PVector.undef(A.rows)
ctx = be.context(1)
t_end = time.perf_counter() + a.seconds
k = 0
while time.perf_counter() < t_end:
    ctx.sync()
    t0 = time.perf_counter()
    ctx.span_start()
    n = 0
    while time.perf_counter() - t0 < a.window:
        for _ in range(20):
            pamd.mul_(y, A, x)
        n += 20
        ctx.sync()
    ctx.span_stop()
    rec = {"t": round(time.perf_counter() - (t_end - a.seconds), 2), "calls": n, "ms_per_mul": round(ctx.span_ms() / n, 4)}
    if a.probe_every and k % a.probe_every == 0:
        rd, cp = pamd._lib.hbm_probe(0, 1 << 30, 10) if hasattr(pamd._lib, "hbm_probe") else (None, None)
        rec["read_gbs"], rec["copy_gbs"] = rd, cp
    print(json.dumps(rec), flush=True)
    k += 1
