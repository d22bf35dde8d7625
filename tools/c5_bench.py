"""BASELINE config 5 on one GPU: FE27 on a Voronoi ("METIS-like") partition,
all parts on device 0, F64/F32/C128/C64.  Reports mul! time (halo included:
device copies between the parts), algorithmic GB/s over all parts, and the
column-encoding coverage (pattern slices / regular rows) of the parts; each
build also reports the parts' SpMV kernel time (HIP events on the parts'
streams, summed over the parts).

    python tools/c5_bench.py [--n 128] [--parts 8] [--dtypes f64,f32,c128,c64]
                             [--own-streams] [--group 0|1]
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
ap.add_argument("--own-streams", action="store_true", help="a stream pair per part (share_streams=False)")
ap.add_argument("--group", type=int, default=1, help="pa_tune spmv_group: 1 grouped launches (default), 0 per part")
ap.add_argument("--rccl", action="store_true", help="halo over RCCL grouped send/recv (HIPBackend(rccl=True))")
ap.add_argument("--probe", action="store_true",
                help="also report pa_hbm_probe's read rate over the same bytes per launch as one mul!")
ap.add_argument("--tune", default="", help="extra pa_tune knobs, key=value[,key=value]")
a = ap.parse_args()
for kv in filter(None, a.tune.split(",")):
    k, v = kv.split("=")
    pamd._lib.tune(k, int(v))
DT = {"f64": np.float64, "f32": np.float32, "c128": np.complex128, "c64": np.complex64}
be = pamd.HIPBackend(devices=[0], share_streams=not a.own_streams, rccl=a.rccl)
pamd._lib.tune("spmv_group", a.group)
parts = be.get_part_ids(a.parts)
N = (a.n,) * 3
owners = pamd.drivers.voronoi_owners(N, a.parts)
for name in a.dtypes.split(","):
    dtype = DT[name]
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
        Bf = f["value_bytes"] + f["index_bytes"] + f["meta_bytes"] + (f["nrows"] + s.num_hids) * S + f["nrows"] * S \
            + (len(ex.lids_snd.local(p).data) + len(ex.lids_rcv.local(p).data)) * (4 + 2 * S)
        info["format_bytes"] = info.get("format_bytes", 0) + Bf
        for k in ("nslices", "pattern_slices", "delta16_slices", "nrows", "regular_rows", "side_rows"):
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
    for _ in range(10):
        pamd.mul_(y, A, x)
    kt = [c.kernel_times() for c in ctxs]
    for c in ctxs:
        c.set_timing(False)
        c.sync()
    # shared stream pair: every part's events bracket the same grouped launches
    if not a.own_streams and a.group:
        km = kt[0]["interior_ms"] + kt[0]["boundary_ms"]
    else:
        km = sum(t["interior_ms"] + t["boundary_ms"] for t in kt)
    probe = pamd._lib.hbm_probe(0, int(info["format_bytes"]), 20)[0] if a.probe else None
    print(json.dumps({"config": f"C5 FE27 {a.n}^3 Voronoi {a.parts} parts on 1 GPU", "dtype": name, "halo": "rccl" if a.rccl else "device reads", "tune": a.tune,
                      "share_streams": not a.own_streams,
                      "spmv_group": a.group, "format_gbs_all_parts": round(info["format_bytes"] / t / 1e9, 1),
                      "format_gbs_kernels": round(info["format_bytes"] / km / 1e6, 1),
                      "ms_per_mul": round(1e3 * t, 4), "gbs_algorithmic_all_parts": round(B / t / 1e9, 1),
                      "kernel_ms_sum_over_parts": round(km, 4), "gbs_algorithmic_kernels": round(B / km / 1e6, 1),
                      "probe_read_gbs_same_bytes": None if probe is None else round(probe, 1),
                      "kernels_of_probe": None if probe is None else round(info["format_bytes"] / km / 1e6 / probe, 4),
                      "setup_s": round(setup, 2), "format": info}), flush=True)
