"""Does the headline's rate depend on where its buffers land?  In one
process: FE27 256^3 F64 operator A1 timed; then more operators / a large
scratch allocation; then A1 again and a late-built A2.  Prints JSON lines
(ms per mul!, HIP-event span over --reps calls).
    python tools/placement_probe.py [--reps 50]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pamd  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--scratch-gb", type=float, default=40.0)
a = ap.parse_args()
be = pamd.HIPBackend(devices=[0])
parts = be.get_part_ids((1, 1, 1))
ctx = be.context(1)


def build():
    A = pamd.drivers.stencil_operator(parts, (256,) * 3, 27)
    x = pamd.PVector.from_host(pamd.map_parts(lambda s: np.random.default_rng(1).uniform(-1, 1, s.num_lids),
                                              A.cols.partition), A.cols)
    return A, x, pamd.PVector.undef(A.rows)


def timeit(tag, s):
    A, x, y = s
    for _ in range(5):
        pamd.mul_(y, A, x)
    ctx.sync()
    ctx.span_start()
    for _ in range(a.reps):
        pamd.mul_(y, A, x)
    ctx.span_stop()
    print(json.dumps({"step": tag, "ms_per_mul": round(ctx.span_ms() / a.reps, 4)}), flush=True)


s1 = build()
timeit("A1 first", s1)
timeit("A1 again", s1)
junk = torch.empty(int(a.scratch_gb * (1 << 30)), dtype=torch.uint8, device="cuda:0")
junk.fill_(1)
torch.cuda.synchronize()
timeit("A1 with scratch allocated", s1)
s2 = build()
timeit("A2 built after scratch", s2)
del junk
torch.cuda.empty_cache()
timeit("A1 after scratch freed", s1)
timeit("A2 after scratch freed", s2)
s3 = build()
timeit("A3 built last", s3)
timeit("A1 last", s1)
