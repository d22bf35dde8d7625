"""Long-row path (row-length histogram) on one part: a FE27 128³ operator
plus `--nlong` rows of `--len` entries each (random columns).  Reports mul!
time with the long rows in their own kernel (exact order, and the
lane-strided tree), against the same matrix's SELL-only cost estimate."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=128)
ap.add_argument("--nlong", type=int, default=64)
ap.add_argument("--len", type=int, default=200000)
a = ap.parse_args()
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
N = (a.n,) * 3
rows = pamd.prange_cartesian(parts, N)
s = rows.partition.local(1)
i, j, v = pamd.drivers.stencil_entries(27, N, s.lid_to_gid)  # row index into gids, column gids
rng = np.random.default_rng(1)
lr = rng.choice(s.num_lids, a.nlong, replace=False) + 1
I2 = np.repeat(lr, a.len)
J2 = rng.integers(1, s.num_lids + 1, a.nlong * a.len)
V2 = rng.uniform(-1, 1, a.nlong * a.len)
Ii = np.concatenate([np.asarray(i, np.int64) + 1, I2])
Jj = np.concatenate([s.to_lids(j), J2])
Vv = np.concatenate([v, V2])
mk = lambda t: pamd.PData(parts.backend, [1], [t], parts.shape)
t0 = time.perf_counter()
A = pamd.PSparseMatrix.from_coo(mk(Ii), mk(Jj), mk(Vv), rows, rows, ids="local")
setup = time.perf_counter() - t0
info = A.values.local(1).info()
x = pamd.PVector.from_host(pamd.map_parts(lambda t: rng.uniform(-1, 1, t.num_lids), rows.partition), rows)
y = pamd.PVector.undef(rows)
ctx = be.context(1)
out = {"workload": f"FE27 {a.n}^3 + {a.nlong} rows x {a.len} random columns", "setup_s": round(setup, 2),
       "long_rows": info["long_rows"], "long_nnz": info["long_nnz"], "nnz": info["nnz"]}
for exact in (1, 0):
    pamd._lib.tune("long_rows_exact", exact)
    for _ in range(3):
        pamd.mul_(y, A, x)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(20):
        pamd.mul_(y, A, x)
    ctx.sync()
    t = (time.perf_counter() - t0) / 20
    out[f"ms_exact{exact}"] = round(1e3 * t, 4)
    out[f"gbs_exact{exact}"] = round(info["nnz"] * 12 / t / 1e9, 1)
pamd._lib.tune("long_rows_exact", 1)
print(json.dumps(out), flush=True)
