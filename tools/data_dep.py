"""Does the SpMV's rate depend on the VALUES it streams (DRAM/fabric power)?
FE27 256^3 F64 one part, the same matrix and x: assembled values, all
values = 1.0 or a dense-mantissa constant (fillstored!), x = 0 / random;
HIP-event span per mul!, interleaved rounds.  python tools/data_dep.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
A = pamd.drivers.stencil_operator(parts, (256,) * 3, 27)
M = A.values.local(1)
ctx = be.context(1)
xr = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(1).uniform(-1, 1, s.num_lids),
                                           A.cols.partition), A.cols)
x0 = pamd.PVector.from_host(pamd.map_parts(lambda s: np.zeros(s.num_lids), A.cols.partition), A.cols)
y = pamd.PVector.undef(A.rows)


def t(x, reps=30):
    for _ in range(3):
        pamd.mul_(y, A, x)
    ctx.sync()
    ctx.span_start()
    for _ in range(reps):
        pamd.mul_(y, A, x)
    ctx.span_stop()
    return round(ctx.span_ms() / reps, 4)


res = {}
for tag, v in (("assembled", None), ("ones", 1.0), ("dense_mantissa", -0.1234567891234567), ("assembled_again", None)):
    if v is not None:
        pamd.fillstored_(A, v)
    for rnd_i in range(3):
        res.setdefault(tag + "/x_random", []).append(t(xr))
        res.setdefault(tag + "/x_zero", []).append(t(x0))
    if tag == "dense_mantissa":  # rebuild the assembled values
        A = pamd.drivers.stencil_operator(parts, (256,) * 3, 27)
for k, v in res.items():
    print(json.dumps({"case": k, "ms": v, "median": float(np.median(v))}), flush=True)
