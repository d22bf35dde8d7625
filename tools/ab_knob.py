"""Interleaved A/B of pa_tune settings on one problem, in one process
(cdna_hip_programming.md §5.4 rule 24): every variant builds its own copies
of the operator under its knobs (build-time knobs such as spmv_delta16 take
effect), then the variants' mul! loops alternate over several rounds.
Reports per variant the median ms per mul! (wall clock over K calls, copies
rotated so every call streams from HBM), the format bytes and GB/s, and
checks that every variant gives the same bits.

    python tools/ab_knob.py --problem stencil --kind 7 --n 128 --variants "spmv_merge=0|spmv_merge=1"
    python tools/ab_knob.py --problem c5 --n 128 --parts 8 --dtype f32 --variants "spmv_delta16=0|spmv_delta16=1"

With --shared (run-time knobs only) every variant runs on the same operator
copies: separate copies differ in physical placement, which alone moves the
time by up to ~15 % on some boxes (profiles/r03/f/).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402

DT = {"f64": np.float64, "f32": np.float32, "c128": np.complex128, "c64": np.complex64}


def parse(v):
    return [tuple((k, int(x)) for k, x in (kv.split("=") for kv in filter(None, var.split(","))))
            for var in v.split("|")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problem", default="stencil", choices=["stencil", "c5"])
    ap.add_argument("--kind", type=int, default=27)
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--shape", default="1,1,1", help="stencil: Cartesian parts, all on device 0")
    ap.add_argument("--parts", type=int, default=8, help="c5: Voronoi parts")
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--variants", required=True, help="key=v[,key=v]|key=v...")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--label", default="")
    ap.add_argument("--shared", action="store_true",
                    help="run-time knobs only: every variant runs on the SAME operator copies (no allocation/"
                         "placement difference between variants)")
    a = ap.parse_args()
    dtype = DT[a.dtype]
    S = np.dtype(dtype).itemsize
    be = pamd.HIPBackend(devices=[0])
    variants = parse(a.variants)
    if a.problem == "stencil":
        shape = tuple(int(v) for v in a.shape.split(","))
        parts = be.get_part_ids(shape)
        N = tuple(a.n * s for s in shape)
        partition = pamd.drivers.stencil_partition(parts, N, a.kind)
        build = lambda: pamd.drivers.stencil_operator(parts, N, a.kind, dtype, partition=partition)
    else:
        parts = be.get_part_ids(a.parts)
        rows, cols, I, J, V = pamd.drivers.irregular_partition(parts, (a.n,) * 3, 27)
        V = pamd.map_parts(lambda v: pamd.drivers.convert_values(v, dtype), V)
        build = lambda: pamd.PSparseMatrix.from_coo(I, J, V, rows, cols, ids="global")
    ctxs = [be.context(p) for p in parts.part_ids]

    def sync():
        for c in ctxs:
            c.sync()

    def knobs(v):
        return [(k, pamd._lib.tune(k, x)) for k, x in v]

    def restore(prev):
        for k, x in reversed(prev):
            pamd._lib.tune(k, x)

    sets, info = {}, {}
    for vi, v in enumerate(variants):
        if a.shared and vi > 0:
            sets[vi], info[vi] = sets[0], info[0]
            continue
        prev = knobs(v)
        A = build()
        B = 0
        for p in parts.part_ids:
            f = A.values.local(p).info()
            s = A.cols.partition.local(p)
            ns = len(A.cols.exchanger.lids_snd.local(p).data)
            nr = len(A.cols.exchanger.lids_rcv.local(p).data)
            B += f["value_bytes"] + f["index_bytes"] + f["meta_bytes"] + (f["nrows"] + s.num_hids) * S + \
                f["nrows"] * S + (ns + nr) * (4 + 2 * S)
        ncopies = max(1, int(np.ceil(1.0e9 / max(B, 1))))
        cp = [(A, B)] + [(build(), B) for _ in range(ncopies - 1)]
        xs = []
        for Ak, _ in cp:
            x = pamd.PVector.from_host(pamd.map_parts(
                lambda s: (np.random.default_rng(s.part).uniform(-1, 1, s.num_lids)).astype(dtype),
                Ak.cols.partition), Ak.cols)
            xs.append((Ak, x, pamd.PVector.undef(Ak.rows, dtype)))
        sets[vi] = xs
        f0 = A.values.local(parts.part_ids[0]).info()
        info[vi] = {"bytes": B, "copies": ncopies,
                   "format": {k: f0[k] for k in ("nslices", "pattern_slices", "delta16_slices",
                                                 "side_rows") if k in f0}}
        restore(prev)
    times = {vi: [] for vi in range(len(variants))}
    out = {}
    for rnd in range(a.rounds):
        for vi, v in enumerate(variants):
            prev = knobs(v)
            xs = sets[vi]
            for i in range(3):
                pamd.mul_(xs[i % len(xs)][2], xs[i % len(xs)][0], xs[i % len(xs)][1])
            sync()
            t0 = time.perf_counter()
            for i in range(a.steps):
                Ak, x, y = xs[i % len(xs)]
                pamd.mul_(y, Ak, x)
            sync()
            times[vi].append(1e3 * (time.perf_counter() - t0) / a.steps)
            if rnd == 0:
                out[vi] = [t.copy() for t in xs[0][2].to_host().parts]
            restore(prev)
    ref = out[0]
    same = {f"{vi}:{dict(v)}": all(np.array_equal(p, q) for p, q in zip(out[vi], ref))
            for vi, v in enumerate(variants)}
    res = []
    for vi, v in enumerate(variants):
        ms = float(np.median(times[vi]))
        res.append({"knobs": dict(v), "ms_median": round(ms, 5), "ms_all": [round(t, 5) for t in times[vi]],
                    "gbs": round(info[vi]["bytes"] / (ms * 1e-3) / 1e9, 1),
                    "frac": round(info[vi]["bytes"] / (ms * 1e-3) / 1e9 / 8000.0, 4), **info[vi]})
    print(json.dumps({"tool": "ab_knob", "label": a.label, "shared": a.shared, "problem": a.problem,
                      "kind": a.kind, "n": a.n,
                      "dtype": a.dtype, "shape": a.shape if a.problem == "stencil" else a.parts,
                      "same_bits": same, "results": res}))


if __name__ == "__main__":
    main()
