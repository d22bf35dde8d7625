"""Per-kernel A/B of the CG pieces on the 256^3 FE27 operator (one process,
interleaved rounds): mul! vs mul!+dot fused, and the x/r update + norm
fused vs the two broadcasts + norm.  Wall time per op with a device sync."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
A = pamd.drivers.stencil_operator(parts, (n, n, n), 27)
cols = A.cols
mk = lambda seed: pamd.PVector.from_host(pamd.map_parts(
    lambda s: np.random.default_rng(seed).uniform(-1, 1, s.num_lids), cols.partition), cols)
u, c, x, r = mk(1), mk(2), mk(3), mk(4)
ctx = be.context(1)


def timed(f, reps=20):
    f()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    ctx.sync()
    return 1e3 * (time.perf_counter() - t0) / reps


ops = {
    "mul!": lambda: pamd.mul_(c, A, u),
    "mul!+dot (separate)": lambda: (pamd.mul_(c, A, u), pamd.dot(u, c)),
    "mul!+dot (fused)": lambda: pamd.mul_dot_(c, A, u),
    "x+=au; r-=ac; norm (separate)": lambda: (pamd.axpy_(x, 1e-9, u), pamd.axmy_(r, 1e-9, c), pamd.norm(r)),
    "x+=au; r-=ac; norm (fused)": lambda: pamd.cg_update_(x, r, u, c, 1e-9),
    "u = r + b u": lambda: pamd.xpby_(u, r, 1e-9),
    "dot": lambda: pamd.dot(u, c),
    "norm": lambda: pamd.norm(r),
}
res = {k: [] for k in ops}
for rnd in range(4):
    for k, f in ops.items():
        res[k].append(timed(f))
for k in ops:
    print(f"{k:34s} median {np.median(res[k]):.4f} ms  min {np.min(res[k]):.4f}")
