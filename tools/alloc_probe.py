"""Is HBM read rate a property of the allocation?  K device buffers of the
same size, allocated one after the other (hipMalloc through pa_vec_create,
the allocation path of every matrix and vector of the library), each read
by the same streaming kernel (pa_vec reductions: norm over the whole
buffer), the buffers timed in interleaved rounds.  Prints one JSON object:
per buffer its virtual address (and its offsets to 2 MiB / 1 GiB
boundaries) and the median GB/s.

    python tools/alloc_probe.py [--gb 3.5] [--k 6] [--rounds 5] [--reps 20]
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
    ap.add_argument("--gb", type=float, default=3.5)
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    be = pamd.HIPBackend(devices=[0])
    parts = be.get_part_ids(1)
    n = int(a.gb * (1 << 30)) // 8
    rows = pamd.prange_linear(parts, n)
    ctx = be.context(1)
    vecs = []
    for k in range(a.k):
        v = pamd.PVector.undef(rows, np.float64).fill_(1.0 + k)
        vecs.append(v)
    ctx.sync()
    addr = [v.values.parts[0].device_ptr() for v in vecs]
    times = [[] for _ in vecs]
    for _ in range(a.rounds):
        for k, v in enumerate(vecs):
            pamd.norm(v)
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                pamd.norm(v)
            ctx.sync()
            times[k].append((time.perf_counter() - t0) / a.reps)
    res = []
    for k in range(a.k):
        t = float(np.median(times[k]))
        res.append({"k": k, "va": hex(addr[k]), "va_mod_2MiB": addr[k] % (2 << 20), "va_mod_1GiB": addr[k] % (1 << 30),
                    "ms": round(1e3 * t, 4), "gbs": round(n * 8 / t / 1e9, 1)})
    print(json.dumps({"tool": "alloc_probe", "gb": a.gb, "k": a.k, "buffers": res}))


if __name__ == "__main__":
    main()
