"""A/B the SpMV kernel variants (pa_tune knobs) in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24).  Kernel time from HIP events
on the SpMV's stream.  Every variant must give the same bits.

  python tools/ab_spmv.py [--n 256] [--kind 27] [--rounds 5]
                          [--variants flags:unroll:format,...]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=256)
ap.add_argument("--kind", type=int, default=27)
ap.add_argument("--dtype", default="f64")
ap.add_argument("--shape", default="1,1,1", help="parts (all on device 0)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--variants", default="1:8:0,1:8:1,0:8:1,1:4:1",
                help="flags:unroll:format[:lds_bytes],...")
ap.add_argument("--comm-cus", type=int, default=0, help="pa_tune comm_cus before the contexts exist")
ap.add_argument("--copies", type=int, default=1, help="rotate over this many copies of (A, x, y)")
a = ap.parse_args()
pamd._lib.tune("comm_cus", a.comm_cus)
dtype = {"f64": np.float64, "f32": np.float32, "c128": np.complex128, "c64": np.complex64}[a.dtype]

be = pamd.HIPBackend(devices=[0])
shape = tuple(int(v) for v in a.shape.split(","))
parts = be.get_part_ids(shape)
N = tuple(a.n * s for s in shape)
partition = pamd.drivers.stencil_partition(parts, N, a.kind)
sets = []
for c in range(a.copies):  # rotated copies: small operators would otherwise sit in the 256 MB MALL
    A = pamd.drivers.stencil_operator(parts, N, a.kind, dtype, partition=partition)
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids).astype(dtype), A.cols.partition), A.cols)
    sets.append((A, x, pamd.PVector.undef(A.rows, dtype)))
A, x, y = sets[0]
p0 = parts.part_ids[0]
ctx = be.context(p0)
S = np.dtype(dtype).itemsize
B = 0
for p in parts.part_ids:
    f = A.values.local(p).info()
    nh = A.cols.partition.local(p).num_hids
    B += f["value_bytes"] + f["index_bytes"] + f["meta_bytes"] + (f["nrows"] + nh) * S + f["nrows"] * S
variants = [tuple(int(t) for t in v.split(":")) for v in a.variants.split(",")]
variants = [v if len(v) == 4 else v + (0,) for v in variants]
res = {v: [] for v in variants}
ref = None
for rnd in range(a.rounds):
    for v in variants:
        pamd._lib.tune("spmv_flags", v[0])
        pamd._lib.tune("spmv_unroll", v[1])
        pamd._lib.tune("spmv_format", v[2])
        pamd._lib.tune("spmv_lds", v[3])
        for Ak, xk, yk in sets:
            pamd.mul_(yk, Ak, xk)
        ctx.sync()
        ctx.span_start()
        for i in range(a.reps):
            Ak, xk, yk = sets[i % a.copies]
            pamd.mul_(yk, Ak, xk)
        ctx.span_stop()
        res[v].append(ctx.span_ms() / a.reps)
        out = y.to_host().local(p0)
        if ref is None:
            ref = out
        assert np.array_equal(out, ref), f"variant {v} changed the result"
print(f"n={a.n} kind={a.kind} dtype={a.dtype} parts={shape} copies={a.copies} part {p0}: {A.values.local(p0).info()}")
print(f"bytes per mul! (format, all parts, current encoding of the last variant) = {B}")
for v in variants:
    t = np.array(res[v])
    print(f"flags={v[0]} unroll={v[1]} format={'pattern' if v[2] else 'int32'} lds={v[3]}: median {np.median(t):.4f} ms "
          f"min {t.min():.4f} -> {B / np.median(t) / 1e6:.0f} GB/s (median), {B / t.min() / 1e6:.0f} (best)")
