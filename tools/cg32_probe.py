"""Float32 CG: the device's residual history against the oracle's Float32
cg! with Julia's scalar typing (Float64 β, α) and with Float32 scalars —
per iteration relative differences (which semantics the device follows)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import pamd  # noqa: E402
import pa_oracle as O  # noqa: E402

shape = (2, 2, 2)
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids(shape)
A, b, x0, _ = pamd.drivers.fdm_problem(parts, 10, np.float32)
x = x0.copy()
hist = []
pamd.cg_(x, A, b, history=hist, device=True)
OA, ob, ox0, _ = O.fdm_problem(O.get_part_ids(shape), 10)
vals = O.map_parts(lambda M: O.CSC(M.m, M.n, M.colptr, M.rowval, O._convert_values(M.nzval, np.float32)), OA.values)
OA32 = O.PSparseMatrix(vals, OA.rows, OA.cols)


def run(f32_scalars):
    ob32 = O.PVector(O.map_parts(lambda v: np.asarray(v, np.float32).copy(), ob.values), ob.rows)
    ox = O.PVector(O.map_parts(lambda v: np.asarray(v, np.float32).copy(), ox0.values), ox0.rows)
    if f32_scalars:
        orig = O.np.float64
        O.np.float64 = np.float32  # the oracle's β, α as Float32 (the pre-round-2 semantics)
    try:
        h = []
        O.cg_(ox, OA32, ob32, log=h)
    finally:
        if f32_scalars:
            O.np.float64 = orig
    return h


hj, hf = run(False), run(True)
for k, (d, a, c) in enumerate(zip(hist, hj, hf)):
    print(f"it {k + 1:3d}  device {d:.9e}  julia-scalars rel {abs(d - a) / a:.2e}  f32-scalars rel {abs(d - c) / c:.2e}")
