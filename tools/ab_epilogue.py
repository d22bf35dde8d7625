"""Interleaved A/B of spmv_flags bit 10 (the fused dot's / fused CG's
epilogue operands loaded before the row loop) on one FE27 256³ operator:
mul! + dot (the CG's SpMV, pamd.mul_dot_) and the device-CG steady state
(cg! of 3K minus cg! of K iterations, u update fused and as a sweep), in
rounds, every variant on the same operator and vectors.  Prints one JSON
object with the medians and whether the results are bit-identical.

    python tools/ab_epilogue.py [--n 256] [--k 10] [--rounds 4] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    be = pamd.HIPBackend(devices=[0])
    parts = be.get_part_ids((1, 1, 1))
    ctx = be.context(1)
    A = pamd.drivers.stencil_operator(parts, (a.n,) * 3, 27)
    mk = lambda seed: pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(seed).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
    u, b = mk(1), mk(2)
    c = pamd.PVector.undef(A.rows)
    base = pamd._lib.tune("spmv_flags", 0)
    pamd._lib.tune("spmv_flags", base)
    variants = {"late": base & ~1024, "early": base | 1024}
    res = {k: {"mul_dot_ms": [], "cg_fused_ms": [], "cg_sweep_ms": []} for k in variants}
    out = {}

    def cg(k, fuse):
        prev = pamd._lib.tune("cg_fuse", fuse)
        x = pamd.PVector.undef(A.cols).fill_(0)
        hist = []
        ctx.sync()
        t0 = time.perf_counter()
        pamd.cg_(x, A, b, reltol=0.0, maxiter=k, history=hist, device=True, batch=16)
        ctx.sync()
        el = time.perf_counter() - t0
        pamd._lib.tune("cg_fuse", prev)
        return el, hist

    for _ in range(a.rounds):
        for name, fl in variants.items():
            pamd._lib.tune("spmv_flags", fl)
            d = pamd.mul_dot_(c, A, u)
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                d = pamd.mul_dot_(c, A, u)
            ctx.sync()
            res[name]["mul_dot_ms"].append(1e3 * (time.perf_counter() - t0) / a.reps)
            for fuse, key in ((1, "cg_fused_ms"), (0, "cg_sweep_ms")):
                e1, h1 = cg(a.k, fuse)
                e3, h3 = cg(3 * a.k, fuse)
                res[name][key].append(1e3 * (e3 - e1) / (len(h3) - len(h1)))
                out[(name, key)] = h3[-1]
            out[(name, "dot")] = d
    pamd._lib.tune("spmv_flags", base)
    same = all(out[("late", k)] == out[("early", k)] for k in ("dot", "cg_fused_ms", "cg_sweep_ms"))
    print(json.dumps({"tool": "ab_epilogue", "n": a.n, "same_results": same,
                      "median": {v: {k: round(float(np.median(t)), 4) for k, t in r.items()} for v, r in res.items()},
                      "all": {v: {k: [round(x, 4) for x in t] for k, t in r.items()} for v, r in res.items()}}))


if __name__ == "__main__":
    main()
