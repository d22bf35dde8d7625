"""Why is the first operator of a process slower than the ones built after
it (profiles/r03/g, profiles/r03/i)?  In a fresh process: optionally touch
and release a device scratch of --prealloc-gb first (or keep it allocated
with --keep), then build K copies of the one-part FE27 256³ operator and
time them in interleaved rounds (HIP events, one x/y pair).

    python tools/first_alloc_probe.py [--prealloc-gb 0] [--keep] [--k 2]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--prealloc-gb", type=float, default=0.0)
    ap.add_argument("--keep", action="store_true")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--swap", action="store_true", help="free the first copy, then build one more")
    ap.add_argument("--dummy-first", type=int, default=0, help="build (and keep) an n^3 operator first")
    ap.add_argument("--tune", default="", help="pa_tune knobs before anything is built: key=v[,key=v]")
    a = ap.parse_args()
    for kv in filter(None, a.tune.split(",")):
        k, v = kv.split("=")
        pamd._lib.tune(k, int(v))
    be = pamd.HIPBackend(devices=[0])
    parts = be.get_part_ids((1, 1, 1))
    ctx = be.context(1)
    scratch = None
    if a.prealloc_gb > 0:
        import torch
        scratch = torch.empty(int(a.prealloc_gb * (1 << 30)), dtype=torch.uint8, device="cuda:0")
        scratch.fill_(7)
        torch.cuda.synchronize()
        if not a.keep:
            del scratch
            scratch = None
            torch.cuda.empty_cache()
    dummy = None
    if a.dummy_first:
        dummy = pamd.drivers.stencil_operator(parts, (a.dummy_first,) * 3, 27, np.float64)
    N = (a.n,) * 3
    partition = pamd.drivers.stencil_partition(parts, N, 27)
    As = [pamd.drivers.stencil_operator(parts, N, 27, np.float64, partition=partition) for _ in range(a.k)]
    if a.swap:
        del As[0]
        As.append(pamd.drivers.stencil_operator(parts, N, 27, np.float64, partition=partition))
    A = As[0]
    x = pamd.PVector.from_host(pamd.map_parts(
        lambda s: np.random.default_rng(s.part).uniform(-1, 1, s.num_lids), A.cols.partition), A.cols)
    y = pamd.PVector.undef(A.rows)
    ctx.sync()
    t = [[] for _ in As]
    for _ in range(a.rounds):
        for i, Ai in enumerate(As):
            pamd.mul_(y, Ai, x)
            ctx.sync()
            ctx.span_start()
            for _ in range(a.reps):
                pamd.mul_(y, Ai, x)
            ctx.span_stop()
            t[i].append(ctx.span_ms() / a.reps)
    ptrs = [{k: hex(v) for k, v in Ai.values.local(1).device_ptrs().items()} for Ai in As]
    print(json.dumps({"tool": "first_alloc_probe", "tune": a.tune, "prealloc_gb": a.prealloc_gb, "keep": a.keep,
                      "swap": a.swap, "dummy_first": a.dummy_first, "mat_ptrs": ptrs,
                      "x": hex(x.values.parts[0].device_ptr()), "y": hex(y.values.parts[0].device_ptr()),
                      "ms": [round(float(np.median(v)), 4) for v in t]}))


if __name__ == "__main__":
    main()
