"""BASELINE config 5 on one GPU: FE27 on a Voronoi ("METIS-like") partition,
all parts on device 0, F64/F32/C128/C64.  Reports mul! time (halo included:
device copies between the parts), algorithmic GB/s over all parts, and the
column-encoding coverage (pattern slices / regular rows) of the parts.
--patterns A/Bs the offset patterns per slice (pa_tune("spmv_patterns"),
1 = single-pattern slices); each build also reports the parts' SpMV kernel
time (HIP events on the parts' streams, summed over the parts).

    python tools/c5_bench.py [--n 128] [--parts 8] [--dtypes f64,f32,c128,c64] [--patterns 1,4] [--share]
"""
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
ap.add_argument("--parts", type=int, default=8)
ap.add_argument("--dtypes", default="f64,f32,c128,c64")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--patterns", default="4")
ap.add_argument("--rules", default="1", help="pa_tune spmv_pattern_rule values to A/B")
ap.add_argument("--share", action="store_true", help="parts as one in-order chain (share_streams)")
ap.add_argument("--graph", action="store_true", help="also time the HIP-graph replay (pamd.SpMVGraph)")
a = ap.parse_args()
DT = {"f64": np.float64, "f32": np.float32, "c128": np.complex128, "c64": np.complex64}
be = pamd.HIPBackend(devices=[0], share_streams=a.share)
parts = be.get_part_ids(a.parts)
N = (a.n,) * 3
owners = pamd.drivers.voronoi_owners(N, a.parts)
for name, npat, rule in [(d, int(q), int(r)) for d in a.dtypes.split(",") for q in a.patterns.split(",")
                         for r in a.rules.split(",")]:
    dtype = DT[name]
    pamd._lib.tune("spmv_patterns", npat)
    pamd._lib.tune("spmv_pattern_rule", rule)
    t0 = time.perf_counter()
    A = pamd.drivers.irregular_problem(parts, N, 27, dtype, owners=owners)
    setup = time.perf_counter() - t0
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids).astype(dtype), A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows, dtype)
    S = np.dtype(dtype).itemsize
    B = 0
    info = {}
    for p in parts.part_ids:
        f = A.values.local(p).info()
        s = A.cols.partition.local(p)
        ex = A.cols.exchanger
        B += (f["nnz"] * (S + 4) + (f["nrows"] + 1) * 4 + (f["nrows"] + s.num_hids) * S + f["nrows"] * S
              + (len(ex.lids_snd.local(p).data) + len(ex.lids_rcv.local(p).data)) * (4 + 2 * S))
        for k in ("nslices", "pattern_slices", "multi_pattern_slices", "nrows", "regular_rows", "side_rows"):
            info[k] = info.get(k, 0) + f[k]
    for _ in range(3):
        pamd.mul_(y, A, x)
    for p in parts.part_ids:
        be.context(p).sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        pamd.mul_(y, A, x)
    for p in parts.part_ids:
        be.context(p).sync()
    t = (time.perf_counter() - t0) / a.steps
    ctxs = [be.context(p) for p in parts.part_ids]
    for c in ctxs:
        c.set_timing(True)
    kms = []
    for _ in range(5):
        pamd.mul_(y, A, x)
        kms.append(sum(sum(c.last_kernel_ms()) for c in ctxs))
    for c in ctxs:
        c.set_timing(False)
        c.sync()
    km = float(np.median(kms))
    t_graph = None
    if a.graph:
        ref = y.to_host()
        g = pamd.SpMVGraph(y, A, x)
        for _ in range(3):
            g()
        for p in parts.part_ids:
            be.context(p).sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            g()
        for p in parts.part_ids:
            be.context(p).sync()
        t_graph = (time.perf_counter() - t0) / a.steps
        got = y.to_host()
        for p in parts.part_ids:
            own = A.rows.partition.local(p).oid_to_lid - 1
            assert np.array_equal(got.local(p)[own], ref.local(p)[own]), "graph replay differs from eager mul!"
        del g
    print(json.dumps({"config": f"C5 FE27 {a.n}^3 Voronoi {a.parts} parts on 1 GPU", "dtype": name,
                      "spmv_patterns": npat, "spmv_pattern_rule": rule, "share_streams": a.share,
                      "ms_per_mul": round(1e3 * t, 4),
                      "ms_per_mul_graph": None if t_graph is None else round(1e3 * t_graph, 4), "gbs_algorithmic_all_parts": round(B / t / 1e9, 1),
                      "kernel_ms_sum_over_parts": round(km, 4), "gbs_algorithmic_kernels": round(B / km / 1e6, 1),
                      "setup_s": round(setup, 2), "format": info}), flush=True)
