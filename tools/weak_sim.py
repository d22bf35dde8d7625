"""Weak-scaling rehearsal on ONE GPU: the 8 parts of BASELINE config 3/4's
(2,2,2) partition (256³ nodes per part, 512³ global) all on device 0, in one
process (halo = device copies).  Reports, per part, the device time of its
SpMV kernels (HIP events on its stream, measured with the other parts idle,
one part at a time) against the same-size single part (1,1,1), i.e. the
extra work a part of the 8-GPU run does (boundary slices, side rows, pack/
unpack) — the part of weak-scaling efficiency that is not RCCL latency.

    python tools/weak_sim.py [--n 256] [--reps 10]

Each part alone is timed through the per-part launches (pa_tune spmv_group
0), which split it into the interior phase (no ghost column: what overlaps
the halo transport on 8 GPUs) and the boundary phase: the interior time is
the per-part halo budget.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
be = pamd.HIPBackend(devices=[0])
out = {}
for shape in ((1, 1, 1), (2, 2, 2)):
    parts = be.get_part_ids(shape)
    N = tuple(a.n * s for s in shape)
    A = pamd.drivers.stencil_operator(parts, N, 27)
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    ctxs = [be.context(p) for p in parts.part_ids]
    for _ in range(3):
        pamd.mul_(y, A, x)
    for c in ctxs:
        c.sync()
    # whole mul! (all parts, halo included) wall time
    import time
    t0 = time.perf_counter()
    for _ in range(a.reps):
        pamd.mul_(y, A, x)
    for c in ctxs:
        c.sync()
    wall = (time.perf_counter() - t0) / a.reps
    # per part device time: time part p alone (mul! on the one-part view is
    # not possible, so time all parts with timing on and read each stream)
    per = {p: [] for p in parts.part_ids}
    for c in ctxs:
        c.set_timing(True)
    for _ in range(a.reps):
        pamd.mul_(y, A, x)
        for p, c in zip(parts.part_ids, ctxs):
            per[p].append(sum(c.last_kernel_ms()))
    for c in ctxs:
        c.set_timing(False)
    # each part ALONE (no halo, other parts idle): what one GPU of the
    # 8-GPU run computes per step, apart from the exchange
    import ctypes as C
    alone = {}
    for p in parts.part_ids:
        c = be.context(p)
        ix = pamd.device.device_index(c, A.cols.partition.local(p))
        iy = pamd.device.device_index(c, A.rows.partition.local(p))
        one, zero = pamd._lib.scalar_buf(1.0, np.float64), pamd._lib.scalar_buf(0.0, np.float64)
        args = (1, pamd._lib.ptr_array([A.values.local(p).h]), pamd._lib.ptr_array([y.values.local(p).h]),
                pamd._lib.ptr_array([iy.h]), pamd._lib.ptr_array([x.values.local(p).h]), pamd._lib.ptr_array([ix.h]),
                None, one[1], zero[1])
        # per-part launches (spmv_group 0): the interior phase (slices
        # without ghost columns: what runs while the halo is in flight on
        # 8 GPUs) and the boundary phase (slices reading ghosts, side rows)
        prev = pamd._lib.tune("spmv_group", 0)
        c.set_timing(True)
        ks, ki, kb = [], [], []
        for _ in range(a.reps + 2):
            pamd._lib.call("pa_spmv_all", *args)
            t = c.kernel_times()
            ks.append(t["interior_ms"] + t["boundary_ms"])
            ki.append(t["interior_ms"])
            kb.append(t["boundary_ms"])
        c.set_timing(False)
        pamd._lib.tune("spmv_group", prev)
        alone[p] = {"total_ms": round(float(np.median(ks[2:])), 4), "interior_ms": round(float(np.median(ki[2:])), 4),
                    "boundary_ms": round(float(np.median(kb[2:])), 4)}
    infos = {p: A.values.local(p).info() for p in parts.part_ids}
    out[str(shape)] = {"wall_ms_per_mul_all_parts": round(1e3 * wall, 4),
                       "wall_ms_per_part": round(1e3 * wall / len(parts.part_ids), 4),
                       "kernel_ms_per_part_median": {p: round(float(np.median(v)), 4) for p, v in per.items()},
                       "kernel_ms_part_alone": alone,
                       "side_rows": {p: infos[p]["side_rows"] for p in parts.part_ids},
                       "ghosts": {p: A.cols.partition.local(p).num_hids for p in parts.part_ids}}
    del A, x, y
print(json.dumps(out), flush=True)
